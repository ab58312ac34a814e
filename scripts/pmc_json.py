"""profiles/pmc_c2.json from the FETCH_SIZE / WRITE_SIZE rocprofv3 passes:
per-launch HBM bytes of one kernel = FETCH_SIZE x F + WRITE_SIZE, KB x 1024,
median over the profiled launches. F = 2 for coalesced streaming reads
(gfx950 under-reports them by half, MI355X_MICROARCH.md HBM section); F = 1
for scattered record loads: scripts/microbench/fetch_calib (profiles/r04/s13/
calib*) measured FETCH_SIZE = 2099 MiB for 33.5 M random 12-byte record loads
(33.5 M x 64-byte fetches = 2048 MiB, x1.02) and 256 MiB for a 512 MiB
16-byte streaming read (x2). Both readings are written.
    python scripts/pmc_json.py <fetch dir> <write dir> <kernel substring> <out.json> [config] [n] [F]"""
import csv
import glob
import json
import statistics
import sys


NAMES = set()


def per_launch(d, counter, kern):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
                kn = r["Kernel_Name"]
                NAMES.add(kn[kn.index(kern):].split("(")[0].strip())
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id") or len(vals))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fd, wd, kern, out = sys.argv[1:5]
    config = sys.argv[5] if len(sys.argv) > 5 else "c2"
    n = int(sys.argv[6]) if len(sys.argv) > 6 else 1000
    fx = float(sys.argv[7]) if len(sys.argv) > 7 else 2.0
    f = statistics.median(per_launch(fd, "FETCH_SIZE", kern))
    w = statistics.median(per_launch(wd, "WRITE_SIZE", kern))
    # the kernel's own (template) name when one instantiation ran, so that
    # bench.py quotes the counters only beside the kernel they were taken on
    kname = next(iter(NAMES)) if len(NAMES) == 1 else kern
    res = {"config": config, "n": n, "kernel": f"{kname} (per launch, median over the profiled launches)",
           "fetch_size_kb": f, "write_size_kb": w,
           "correction": (f"FETCH_SIZE x{fx:g} + WRITE_SIZE, x1024 B/KB (x2: coalesced streaming reads, "
                          "MI355X_MICROARCH.md HBM section; x1: scattered record loads, "
                          "scripts/microbench/fetch_calib, profiles/r04/s13/calib*)"),
           "hbm_bytes_per_launch": (fx * f + w) * 1024.0,
           "hbm_bytes_x1": (f + w) * 1024.0, "hbm_bytes_x2": (2 * f + w) * 1024.0,
           "source": f"{fd}, {wd}"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
