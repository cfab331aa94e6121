#!/bin/bash
# Round 3: listed GPU tests, filter-only bench lines of chain modes, pass_bench of C3 with an optional
# C' diagnostic mask.  Usage (GPU box): TAG "tests..." "modes..." [DIAG]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3q}; mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $2 > $O/tests.log 2>&1
  rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -30 | cut -c1-300; exit $rc; }
fi
for ch in $3; do
  timeout -k 10 300 python3 bench.py --filter-only --chain $ch --steps 20 --warmup 3 --no-cpu-baseline > $O/filter_$ch.json 2> $O/filter_$ch.err || { echo "$ch failed"; tail -5 $O/filter_$ch.err; exit 1; }
  python3 -c "
import json; l=json.loads(open('$O/filter_$ch.json').read().strip().splitlines()[-1])
print('$ch', l['value'], l['filter_ms_per_step'], {k:(v['kernel'],v['avg_ms'],v.get('GB_s')) for k,v in l['filter_passes'].items()})"
done
timeout -k 10 300 python3 scripts/pass_bench.py --config c3 --iters 30 --flush-mb 0 > $O/pass.txt 2>&1 && tail -6 $O/pass.txt || { tail -5 $O/pass.txt; exit 1; }
if [ -n "$4" ]; then
  TEXBIAS_BAND_DIAG=$4 timeout -k 10 300 python3 scripts/pass_bench.py --config c3 --iters 30 --flush-mb 0 > $O/pass_diag.txt 2>&1 && tail -6 $O/pass_diag.txt || { tail -5 $O/pass_diag.txt; exit 1; }
fi
echo done
