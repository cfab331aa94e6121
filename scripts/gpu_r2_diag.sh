#!/bin/bash
# Stage attribution of the band passes: filter-only bench per TEXBIAS_BAND_DIAG mask (results invalid
# in the masked runs; timing only).  Usage: bash scripts/gpu_r2_diag.sh TAG MASK...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2d}; shift
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_fusedchain.py > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for m in 0 "$@"; do
  TEXBIAS_BAND_DIAG=$m timeout -k 10 120 python bench.py --filter-only --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$T/b_$m.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$T/b_$m.json').read().strip().splitlines()[-1]); p=d['filter_passes']; print('$m', {k:(v['kernel'],v['avg_ms']) for k,v in p.items()})"
done
