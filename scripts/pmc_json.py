"""profiles/pmc_c2.json from the FETCH_SIZE / WRITE_SIZE rocprofv3 passes:
per-launch HBM bytes of one kernel = FETCH_SIZE x 2 (gfx950 under-reports
wide streaming reads by half, MI355X_MICROARCH.md HBM section) + WRITE_SIZE,
KB x 1024, median over the profiled launches.
    python scripts/pmc_json.py <fetch dir> <write dir> <kernel substring> <out.json> [config] [n]"""
import csv
import glob
import json
import statistics
import sys


def per_launch(d, counter, kern):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id") or len(vals))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fd, wd, kern, out = sys.argv[1:5]
    config = sys.argv[5] if len(sys.argv) > 5 else "c2"
    n = int(sys.argv[6]) if len(sys.argv) > 6 else 1000
    f = statistics.median(per_launch(fd, "FETCH_SIZE", kern))
    w = statistics.median(per_launch(wd, "WRITE_SIZE", kern))
    res = {"config": config, "n": n, "kernel": f"{kern} (per launch, median over the profiled launches)",
           "fetch_size_kb": f, "write_size_kb": w,
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, x1024 B/KB",
           "hbm_bytes_per_launch": (2 * f + w) * 1024.0, "source": f"{fd}, {wd}"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
