#!/usr/bin/env python3
"""Average PMC counter values per kernel from rocprofv3 --pmc runs (one dir per pass).
Usage: pmc_summary.py DIR [DIR ...]   (each DIR holds */run_counter_collection.csv)"""
import collections
import csv
import glob
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)<([^>]*)>", r["Kernel_Name"]) or re.search(r"(k_\w+)", r["Kernel_Name"])
            k = m.group(0) if m else r["Kernel_Name"][:40]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {sum(x) / len(x):16.1f}   (n={len(x)})")
