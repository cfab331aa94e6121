#!/bin/bash
# timing-only A/B of library variants with the stage-skip diag masks: bash scripts/gpu_ab_diag.sh TAG MASK lib...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; M=$2; shift 2
mkdir -p gpurun_out/$T
i=0
for v in default "$@"; do
  for m in 0 $M; do
    if [ "$v" = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=$PWD/$v; fi
    TEXBIAS_BAND_DIAG=$m timeout -k 10 120 python bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/$T/b_$i.json 2>/dev/null || { echo "bench $v $m failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$T/b_$i.json').read().strip().splitlines()[-1]); p=d['filter_passes']; print('$v', '$m', p['inverse']['avg_ms'])"
    i=$((i+1))
  done
done
