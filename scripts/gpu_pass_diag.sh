#!/bin/bash
# Stage attribution of the band passes with scripts/pass_bench.py per TEXBIAS_BAND_DIAG mask
# (results invalid in masked runs; timing only).  Usage: bash scripts/gpu_pass_diag.sh TAG MASK...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-pdiag}; shift
mkdir -p gpurun_out/$T
for m in 0 "$@"; do
  for cfg in ${PB_CONFIGS:-c3}; do
    TEXBIAS_BAND_DIAG=$m timeout -k 10 120 python scripts/pass_bench.py --config $cfg --iters ${PB_ITERS:-40} --tag diag$m ${PB_ARGS:---flush-mb 0} 2>gpurun_out/$T/err.txt || { echo "diag $m failed"; tail -5 gpurun_out/$T/err.txt; exit 1; }
  done
done
