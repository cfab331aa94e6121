#!/usr/bin/env python3
"""HBM traffic per launch of the filter kernels from two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE),
corrected per MI355X_MICROARCH.md (gfx950 FETCH_SIZE = half the bytes of a wide streaming read).
Usage: make_traffic.py FETCH_DIR WRITE_DIR BENCH_FILTER_JSON OUT.json
The bench line (bench.py --filter-only, same launch shapes) supplies each kernel's algorithmic
bytes per launch, which bench.py matches against before it reports `roofline.traffic`."""
import collections
import csv
import glob
import json
import re
import sys


def read(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            if m:
                vals[m.group(1)].append(float(r["Counter_Value"]) * 1024.0)  # KiB -> bytes
    return vals


fetch = read(sys.argv[1], "FETCH_SIZE")
write = read(sys.argv[2], "WRITE_SIZE")
bench = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
alg = {p["kernel"]: p.get("algorithmic_bytes") for p in bench["filter_passes"].values()}
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, python3 bench.py "
                 + (sys.argv[5] if len(sys.argv) > 5 else "--filter-only") + " ; per-launch averages",
       "correction": "FETCH_SIZE (KiB) x 1024 x 2 per MI355X_MICROARCH.md HBM section (gfx950 tallies 128-B "
                     "requests at 64 B; calibrated there for 16-B/lane reads), WRITE_SIZE (KiB) x 1024 as is",
       "kernels": {}}
for k in sorted(set(fetch) & set(write)):
    f = sum(fetch[k]) / len(fetch[k])
    w = sum(write[k]) / len(write[k])
    out["kernels"][k] = {"launches": len(fetch[k]), "fetch_size_raw_bytes": round(f), "write_size_bytes": round(w),
                         "traffic_bytes": round(2 * f + w), "algorithmic_bytes_per_launch": alg.get(k)}
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out, indent=1))
