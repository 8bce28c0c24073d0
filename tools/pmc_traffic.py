"""HBM traffic per launch from rocprofv3 --pmc passes (FETCH_SIZE pass + WRITE_SIZE pass).

MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read, so

    traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   bytes per dispatch

(mean over the dispatches of each kernel; counters summed over the dimensions rocprofv3
splits them into).  Writes a JSON {kernel_key: {"fetch_kib", "write_kib", "traffic_bytes",
"dispatches"}} that bench.py reads for the "traffic" field.

    python tools/pmc_traffic.py OUT.json FETCH_pass.csv WRITE_pass.csv
"""
import csv
import json
import sys
from collections import defaultdict

KEYS = {"k_gen": "k_gen<", "k_cons": "k_cons<", "k_genc": "k_genc<", "k_narrow": "k_narrow<",
        "k_mlp": ("k_mlp2<", "k_mlpr<"), "k_survive": "k_survive<"}


def per_dispatch(paths, counter):
    tot = defaultdict(lambda: defaultdict(float))
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                for key, pat in KEYS.items():
                    pats = pat if isinstance(pat, tuple) else (pat,)
                    if any(q in r["Kernel_Name"] for q in pats):
                        tot[key][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in tot.items() if v}


def main(out, *paths):
    fetch = per_dispatch(paths, "FETCH_SIZE")
    write = per_dispatch(paths, "WRITE_SIZE")
    res = {}
    for k in KEYS:
        if k in fetch and k in write:
            f, n = fetch[k]
            w, _ = write[k]
            res[k] = {"fetch_kib": f, "write_kib": w, "traffic_bytes": (2 * f + w) * 1024,
                      "dispatches": n}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
