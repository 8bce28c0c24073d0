"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin) per kernel."""
import re
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat in r["name"]:
        print(f'{r["name"][:40]:40s} vgpr={r.get("VGPRs")} agpr={r.get("AGPRs")} '
              f'occ={r.get("Occupancy [waves/SIMD]")} sspill={r.get("SGPRs Spill")} '
              f'vspill={r.get("VGPRs Spill")}')
