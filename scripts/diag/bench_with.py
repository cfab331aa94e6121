#!/usr/bin/env python3
"""bench.py with texbias module constants overridden (measurement tool, A/B of routing thresholds):
    python3 scripts/diag/bench_with.py conv.MIN_K_PER_OUTPUT=1 -- --steps 10 --no-cpu-baseline"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
i = sys.argv.index("--")
sets, args = sys.argv[1:i], sys.argv[i + 1:]
import importlib  # noqa: E402
for kv in sets:
    k, v = kv.split("=")
    mod, attr = k.rsplit(".", 1)
    m = importlib.import_module("texbias." + mod)
    old = getattr(m, attr)
    setattr(m, attr, type(old)(eval(v)))
    print(f"[bench_with] texbias.{k}: {old} -> {getattr(m, attr)}", file=sys.stderr)
sys.argv = [os.path.join(ROOT, "bench.py")] + args
runpy.run_path(sys.argv[0], run_name="__main__")
