#!/usr/bin/env python3
"""HBM traffic per launch of the filter passes from two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE),
corrected per MI355X_MICROARCH.md (gfx950 FETCH_SIZE = half the bytes of a wide streaming read).
Usage: make_traffic.py FETCH_DIR WRITE_DIR OUT.json  -- launches of bench.py --filter-only (C3, B=2)."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import algorithmic_bytes  # noqa: E402

NAMES = (("k_slab_fwd_ct", "slab_fwd"), ("k_kspace_ct", "kspace"), ("k_slab_inv_ct", "slab_inv"))


def read(d, counter):
    vals, kname = collections.defaultdict(list), {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for pre, nm in NAMES:
                if pre in r["Kernel_Name"]:
                    vals[nm].append(float(r["Counter_Value"]) * 1024.0)  # KiB -> bytes
                    kname[nm] = r["Kernel_Name"]
    return vals, kname


fetch, kn = read(sys.argv[1], "FETCH_SIZE")
write, _ = read(sys.argv[2], "WRITE_SIZE")
alg = algorithmic_bytes(8, 240, 240, 155, 5)
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, python3 bench.py --filter-only "
                 "(B=2 x 4 x 240x240x155, output padded to 160); per-launch averages",
       "correction": "FETCH_SIZE (KiB) x 1024 x 2 per MI355X_MICROARCH.md HBM section (gfx950 tallies 128-B "
                     "requests at 64 B; calibrated there for 16-B/lane reads), WRITE_SIZE (KiB) x 1024 as is",
       "kernels": {}}
for _, nm in NAMES:
    if fetch.get(nm) and write.get(nm):
        f = sum(fetch[nm]) / len(fetch[nm])
        w = sum(write[nm]) / len(write[nm])
        out["kernels"][nm] = {"kernel": kn[nm], "launches": len(fetch[nm]), "fetch_size_raw_bytes": round(f),
                              "write_size_bytes": round(w), "traffic_bytes": round(2 * f + w),
                              "algorithmic_bytes_per_launch": alg[nm]}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
