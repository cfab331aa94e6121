#!/usr/bin/env python3
"""Per-kernel summary of the LAST `--steps` bench steps of a rocprofv3 kernel trace.

A step is delimited by the filter's first pass (k_slab_fwd); the summary covers the window
from the (steps)-th-last k_slab_fwd launch to the end of the trace, so MIOpen's Find phase
and the warmup steps are excluded.  Usage: steady_stats.py run_kernel_trace.csv --steps K
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--marker", default="k_slab_fwd")
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--per-step", type=int, default=1, help="marker launches per step")
ap.add_argument("--calls", default=None, help="also list the last step's launches whose name matches this regex")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"]]
t0 = starts[-a.steps * a.per_step]
agg = collections.defaultdict(lambda: [0, 0])
t_end = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0:
        continue
    t_end = max(t_end, e)
    nm = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:90]
    agg[nm][0] += 1
    agg[nm][1] += e - s
tot = sum(v[1] for v in agg.values())
print(f"window {(t_end - t0) / 1e6:.2f} ms over {a.steps} steps; kernel busy {tot / 1e6:.2f} ms "
      f"({tot / a.steps / 1e6:.2f} ms/step)")
print(f"{'ms/step':>9} {'%':>6} {'calls/step':>10} {'avg_us':>9}  kernel")
for nm, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
    print(f"{d / a.steps / 1e6:9.3f} {100 * d / tot:6.1f} {n / a.steps:10.1f} {d / n / 1e3:9.1f}  {nm}")

if a.calls:
    last = starts[-a.per_step]
    print(f"\nlast step's launches matching {a.calls!r} (start offset us, duration us, grid, workgroup):")
    for r in rows:
        s = int(r["Start_Timestamp"])
        if s < last or not re.search(a.calls, r["Kernel_Name"]):
            continue
        g = r.get("Grid_Size") or "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        wg = r.get("Workgroup_Size") or "x".join(r.get(k, "?") for k in ("Workgroup_Size_X", "Workgroup_Size_Y",
                                                                          "Workgroup_Size_Z"))
        nm = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:60]
        print(f"{(s - last) / 1e3:10.1f} {(int(r['End_Timestamp']) - s) / 1e3:8.1f}  {g:>14} {wg:>8}  {nm}")
