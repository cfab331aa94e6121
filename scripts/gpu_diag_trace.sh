#!/bin/bash
# rocprofv3 kernel durations of the filter passes per TEXBIAS_BAND_DIAG mask (timing only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
for m in 0 "$@"; do
  TEXBIAS_BAND_DIAG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/d$m -o run -- python3 bench.py --filter-only --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || { echo "trace $m failed"; exit 1; }
  echo "== mask $m"; grep -h "k_band\|k_sap" gpurun_out/$T/d$m/run_kernel_stats.csv | awk -F'",' '{print $1}' | head -0
  python3 - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/$T/d$m/run_kernel_stats.csv")):
    n=r["Name"]
    if "k_band" in n or "k_sap" in n or "minmax" in n:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us  {n[:70]}')
PY
done
