#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection CSVs per kernel (average per dispatch): pmc_kernel.py CSV... [--match NAME]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
if match in args:
    args.remove(match)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in args:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        k = k.split("(")[0][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, c in agg.items():
    n = len(disp[k])
    print(f"{k}  ({n} dispatches)")
    for name, v in sorted(c.items()):
        print(f"    {name:28s} {v / n:16.1f}")
