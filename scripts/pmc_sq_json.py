"""profiles/pmc_<config>_sq.json from rocprofv3 SQ / TA counter passes: the
per-launch value (median over the profiled launches) of every counter in the
given directories for one kernel. bench.py reads it for the VALU-issue
roofline of that kernel (VALU wave-instructions per launch, per 64 products).
    python scripts/pmc_sq_json.py <out.json> <config> <n> <kernel substring> <dir> [<dir> ...]"""
import csv
import glob
import json
import statistics
import sys


def main():
    out, config, n, kern = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    dirs = sys.argv[5:]
    vals = {}
    name = None
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            per = {}
            for r in csv.DictReader(open(f)):
                if kern not in r["Kernel_Name"]:
                    continue
                kn = r["Kernel_Name"]
                name = name or kn[kn.index(kern):].split("(")[0]
                key = (r["Counter_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            for (c, _), v in per.items():
                vals.setdefault(c, []).append(v)
    res = {"config": config, "n": n, "kernel": name, "counters_per_launch": {c: statistics.median(v) for c, v in
                                                                          sorted(vals.items())},
           "launches": {c: len(v) for c, v in sorted(vals.items())}, "source": ", ".join(dirs)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
