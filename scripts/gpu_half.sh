#!/bin/bash
# Full-route half units: their GPU tests, then the gibbs-aug chain (filter only, C3 shape) with the half
# units in each launch configuration and with whole slabs, and a rocprofv3 kernel-stats run of the default.
# Usage (GPU box): TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-half}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_half.py tests/test_gpu_kernels.py tests/test_gpu_c4_extremes.py tests/test_gpu_wrap.py tests/test_gpu_point.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
b() {  # name, env..., -- bench args
  local n=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --filter-only --chain gibbs-aug --steps 30 --warmup 5 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$n.json')); print('$n', d['filter_ms_per_step'], {k: (v['kernel'], v['avg_ms'], v.get('GB_s')) for k, v in d['filter_passes'].items()})"
}
b whole TEXBIAS_HALF=0
b half0 TEXBIAS_HALF_CFG=0
b half1 TEXBIAS_HALF_CFG=1
b half2 TEXBIAS_HALF_CFG=2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --filter-only --chain gibbs-aug --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err || { echo prof failed; tail -5 $O/prof.err; exit 1; }
cp $(find $O/prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
rm -f $(find $O/prof -name '*kernel_trace.csv')
head -8 $O/kernel_stats.csv | cut -c1-200
echo done
