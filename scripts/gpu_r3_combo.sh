#!/bin/bash
# Round 3: C' sweep (scripts/gpu_r3_inv16_sweep.sh) then the listed GPU test files.
# Usage (GPU box): bash scripts/gpu_r3_combo.sh TAG [test files...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r3c}; shift
bash scripts/gpu_r3_inv16_sweep.sh $T || exit 1
O=gpurun_out/$T
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu "$@" > $O/tests_extra.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|loss texbias|^  model" $O/tests_extra.log | tail -60; [ $rc = 0 ] || { tail -40 $O/tests_extra.log; exit $rc; }
fi
echo done
