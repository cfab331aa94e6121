#!/usr/bin/env python3
"""Per-kernel resource usage of the hot HIP sources (hipcc -Rpass-analysis=kernel-resource-usage, gfx950):
VGPRs, AGPRs, scratch bytes per lane, occupancy (waves per SIMD), static LDS.  Writes a markdown table
(stdout).  Usage: scripts/resource_usage.py [source.hip ...]  (default: every csrc/*.hip with the
Makefile's flags; the full-route slab sources with TB_RS=1)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "medical-vision-textural-bias_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT}/include", f"-I{CSRC}",
         "-Wno-unused-function", "-Wno-unknown-pragmas", "-Rpass-analysis=kernel-resource-usage"]
NOSLP = {"kern_slab_ct.hip", "kern_kspace_ct.hip", "kern_wrap.hip", "kern_band.hip"}
srcs = sys.argv[1:] or sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
rows = []
for src in srcs:
    extra = ["-fno-slp-vectorize"] if src in NOSLP else []
    if src in ("kern_slab_fwd.hip", "kern_slab_inv.hip", "kern_kspace.hip", "kern_stats.hip"):
        extra.append("-DTB_RS=1")
    with tempfile.TemporaryDirectory() as td:
        p = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + extra + ["-c", os.path.join(CSRC, src), "-o",
                                                                        os.path.join(td, "o.o")],
                           capture_output=True, text=True)
    cur = None
    for line in p.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"src": src, "name": m.group(1)}
            rows.append(cur)
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))


def demangle(n):
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


print("| source | kernel | VGPRs | AGPRs | scratch B/lane | waves/SIMD | static LDS B |")
print("|---|---|---|---|---|---|---|")
for r in rows:
    nm = re.sub(r"\(anonymous namespace\)::", "", demangle(r["name"]))
    nm = re.sub(r"\(.*", "", nm).replace("void ", "")
    print(f"| {r['src']} | `{nm}` | {r.get('vgpr', '')} | {r.get('agpr', '')} | {r.get('scratch', '')} | "
          f"{r.get('occ', '')} | {r.get('lds', '')} |")
