#!/bin/bash
# Round-2 GPU check: band-limited pass parity + FusedChain parity, then a filter-only bench.
# Usage (from the repo root, on the GPU box): bash scripts/gpu_r2_check.sh [tag] [pytest selection...]
set -o pipefail
tag=${1:-r2a}
shift
sel=${@:-tests/test_gpu_band.py tests/test_gpu_fusedchain.py tests/test_gpu_kernels.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() {  # a fault / abort / time limit ends the call: nothing more runs on the GPU
  case $1 in 0|1) return 0 ;; *) echo "GPU step failed rc=$1: stopping"; exit "$1" ;; esac
}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $sel \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/${tag}_tests.log; stop $rc
timeout -k 10 300 python -u bench.py --filter-only --steps 20 --warmup 3 --no-cpu-baseline \
  > gpurun_out/${tag}_bench_filter.json 2> gpurun_out/${tag}_bench_filter.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${tag}_bench_filter.json; stop $rc
