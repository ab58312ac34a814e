"""Mean of every PMC counter per kernel (name substring filter) over the
dispatches of rocprofv3 --pmc CSV outputs: python scripts/pmc_summary.py
<dir>... [--kernel NAME]."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = None
    if "--kernel" in sys.argv:
        filt = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != filt]
    vals = defaultdict(list)
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "")
                    if filt and filt not in k:
                        continue
                    vals[(k.split("(")[0][:90], row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in sorted(vals.items()):
        print(f"{k:90s} {c:28s} n={len(v):4d} mean={sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main()
