"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per dispatch,
per kernel (counters summed over the dimensions rocprofv3 splits them into)."""
import csv
import sys
from collections import defaultdict


def main(paths):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                if len(k) > 60:
                    k = k[:60]
                disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k in sorted(tot):
        items = []
        for c, v in sorted(tot[k].items()):
            n = len(disp[(k, c)])
            items.append(f"{c}={v / max(n, 1):.4g}")
        print(k, "|", " ".join(items))


if __name__ == "__main__":
    main(sys.argv[1:])
