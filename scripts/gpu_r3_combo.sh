#!/bin/bash
# Round 3: C' sweep (scripts/gpu_r3_inv16_sweep.sh) then the listed GPU test files.
# Usage (GPU box): bash scripts/gpu_r3_combo.sh TAG [test files...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r3c}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_band.py > $O/tests_band.log 2>&1
rc=$?; grep -cE "PASSED" $O/tests_band.log; [ $rc = 0 ] || { grep -E "Error|assert" $O/tests_band.log | head -30; tail -30 $O/tests_band.log; exit $rc; }
bash scripts/gpu_r3_inv16_sweep.sh $T || exit 1
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu "$@" > $O/tests_extra.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|loss texbias|^  model" $O/tests_extra.log | tail -60; [ $rc = 0 ] || { tail -40 $O/tests_extra.log; exit $rc; }
fi
echo done
