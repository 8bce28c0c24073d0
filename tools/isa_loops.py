"""List the loops of one kernel in a hipcc --save-temps .s file (development tool).

    python tools/isa_loops.py file.s symbol

Prints each backward branch (loop) with the instruction count of its body by class
(v_ VALU, s_ SALU, ds_ LDS, global_/buffer_ memory, v_mfma) -- a quick static view of
where a kernel's instructions are.
"""
import collections
import re
import sys

src, sym = sys.argv[1], sys.argv[2]
s = open(src).read()
i = s.index(sym + ":")
j = s.index(".Lfunc_end", i)
lines = s[i:j].split("\n")
labels, ins = {}, []
for ln in lines:
    m = re.match(r"^(\.LBB\S+):", ln)
    if m:
        labels[m.group(1)] = len(ins)
        continue
    t = ln.strip()
    if ln.startswith("\t") and t and not t.startswith((".", ";")):
        ins.append(t)


def cls(t):
    op = t.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    for p in ("v_", "s_", "ds_", "global_", "buffer_", "scratch_", "flat_"):
        if op.startswith(p):
            return p.rstrip("_")
    return "other"


print(sym, "total", len(ins), dict(collections.Counter(cls(t) for t in ins)))
for k, t in enumerate(ins):
    op = t.split()[0]
    if op.startswith("s_cbranch") or op == "s_branch":
        tgt = t.split()[-1]
        if tgt in labels and labels[tgt] <= k:
            body = ins[labels[tgt]:k + 1]
            c = collections.Counter(cls(x) for x in body)
            f64 = sum(1 for x in body if "_f64" in x.split()[0])
            print(f"loop {tgt} [{labels[tgt]}..{k}] n={len(body)} f64={f64} {dict(c)}")
