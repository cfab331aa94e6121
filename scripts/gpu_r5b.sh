#!/bin/bash
# Round-5 batch: conv tests touched by the in-kernel weight flip and the ConvTranspose3d GEMM input
# gradient, the GEMM-vs-MIOpen layer table, the half-unit C launch config (768 vs 512 threads) on the
# gibbs-aug chain, then the C3 step line + steady breakdown.  Usage (GPU box): TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r5b}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_up.py tests/test_gpu_conv_gemm.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u scripts/diag/gemm_conv_bench.py > $O/gemm.txt 2>&1 || { echo gemm bench failed; tail -20 $O/gemm.txt; exit 1; }
cat $O/gemm.txt
b() {  # name, env...
  local n=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --filter-only --chain gibbs-aug --steps 30 --warmup 5 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['filter_ms_per_step'], {k: (v['kernel'], v['avg_ms'], v.get('GB_s')) for k, v in d['filter_passes'].items()})"
}
b cinv768 TEXBIAS_X=0
b cinv512 TEXBIAS_HALF_CFG_INV=2
bash scripts/gpu_step.sh $T/step || exit 1
echo done
