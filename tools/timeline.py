"""Kernel overlap from a rocprofv3 --kernel-trace CSV (bench.py with its default state groups).

Prints, over the dispatches between the first and last k_survive of the run (steady-state
generations), per kernel: launches, summed duration, mean duration; and for the window: the
wall time, the time with >= 1 kernel running (union), and the mean number of concurrent
kernels.  union / wall near 1 and concurrency near 1 mean the chain is serial; the per-
generation wall divided by the kernels' summed time is the overlap the streams achieve.

    python tools/timeline.py run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

KEYS = {"k_gen": "k_gen<", "k_cons": "k_cons<", "k_genc": "k_genc<", "k_narrow": "k_narrow<",
        "k_mlp": ("k_mlp2<", "k_mlpr<"), "k_mlp2x": "k_mlp2x<", "k_predict": "k_predict<", "k_survive": "k_survive<"}


def key(name):
    for k, p in KEYS.items():
        if any(q in name for q in (p if isinstance(p, tuple) else (p,))):
            return k
    return "other"


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), key(r["Kernel_Name"])))
    rows.sort()
    surv = [r for r in rows if r[2] == "k_survive"]
    if len(surv) < 8:
        print("too few k_survive dispatches", len(surv))
        return
    # skip the first and last 10% of the survival launches (setup, tail)
    lo = surv[len(surv) // 10][0]
    hi = surv[-len(surv) // 10][1]
    win = [r for r in rows if r[0] >= lo and r[1] <= hi and r[2] != "other"]
    per = defaultdict(lambda: [0, 0.0])
    for s, e, k in win:
        per[k][0] += 1
        per[k][1] += (e - s) / 1e3
    ev = sorted([(s, 1) for s, _, _ in win] + [(e, -1) for _, e, _ in win])
    cur, last, union, area = 0, ev[0][0], 0.0, 0.0
    for t, d in ev:
        if cur > 0:
            union += (t - last) / 1e3
            area += cur * (t - last) / 1e3
        cur += d
        last = t
    wall = (hi - lo) / 1e3
    n_surv = per["k_survive"][0]
    print(f"window {wall:.1f} us, {n_surv} k_survive launches")
    tot = 0.0
    for k, (n, us) in sorted(per.items()):
        tot += us
        print(f"  {k:10s} launches {n:6d} sum {us:10.1f} us  mean {us / n:8.2f} us")
    print(f"  busy (>=1 kernel) {union:.1f} us = {union / wall:.3f} of wall; "
          f"mean concurrency while busy {area / max(union, 1e-9):.2f}; "
          f"kernel sum / wall {tot / wall:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
