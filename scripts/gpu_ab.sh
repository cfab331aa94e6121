#!/bin/bash
# A/B of library variants on the filter-only bench: default libtexbias.so, then each .so given.
# Usage: bash scripts/gpu_ab.sh TAG [variant.so ...]   (band tests run on the default first)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_fusedchain.py > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
i=0
for v in default "$@"; do
  if [ "$v" = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=$PWD/$v; fi
  timeout -k 10 120 python bench.py --filter-only --steps ${AB_STEPS:-200} --warmup ${AB_WARM:-30} --no-cpu-baseline > gpurun_out/$T/b_$i.json 2>gpurun_out/$T/b_$i.err || { echo "bench $v failed"; tail -3 gpurun_out/$T/b_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$T/b_$i.json').read().strip().splitlines()[-1]); p=d['filter_passes']; print('$v', {k:(v['kernel'],v['avg_ms']) for k,v in p.items()}, d['filter_ms_per_step'])"
  i=$((i+1))
done
