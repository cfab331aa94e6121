#!/bin/bash
# Per-pass timings (scripts/pass_bench.py) of the default library and each variant .so given.
# Usage: bash scripts/gpu_pass.sh TAG [variant.so ...]   (PB_TESTS=1: band parity tests first, per variant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-pass}; shift
mkdir -p gpurun_out/$T
for v in default "$@"; do
  if [ "$v" = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=$PWD/$v; fi
  if [ -n "$PB_TESTS" ]; then
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_fusedchain.py > gpurun_out/$T/tests_$(basename $v).log 2>&1
    rc=$?; echo "$v tests: $(tail -1 gpurun_out/$T/tests_$(basename $v).log)"; case $rc in 0|1) ;; *) exit $rc ;; esac
  fi
  for cfg in ${PB_CONFIGS:-c3 c2}; do
    timeout -k 10 120 python scripts/pass_bench.py --config $cfg --iters ${PB_ITERS:-40} ${PB_ARGS} 2>gpurun_out/$T/err.txt || { echo "pass_bench $v $cfg failed"; tail -5 gpurun_out/$T/err.txt; exit 1; }
  done
done
