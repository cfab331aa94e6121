#!/bin/bash
# GPU tests (optional), then filter-only bench lines of every chain mode (ref, planes, wrap,
# gibbs-aug, spikes-aug) with a rocprofv3 kernel-trace summary each.  Usage (GPU box): TAG [tests|all|none]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-modes}; mkdir -p $O
if [ "${2:-none}" = all ]; then
  timeout -k 10 800 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests_all.log 2>&1
  rc=$?; tail -3 $O/tests_all.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/tests_all.log | head -20 | cut -c1-300; exit $rc; }
elif [ "${2:-none}" != none ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $2 > $O/tests.log 2>&1
  rc=$?; grep -cE "PASSED" $O/tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -30 | cut -c1-300; exit $rc; }
fi
for ch in ref planes wrap gibbs-aug spikes-aug; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$ch -o run -- python3 bench.py --filter-only --chain $ch --steps 20 --warmup 3 --no-cpu-baseline > $O/filter_$ch.json 2> $O/filter_$ch.err || { echo "$ch failed"; tail -5 $O/filter_$ch.err; exit 1; }
  python3 -c "
import json; l=json.loads(open('$O/filter_$ch.json').read().strip().splitlines()[-1])
print('$ch', l['value'], l['filter_ms_per_step'], {k:(v['kernel'],v['avg_ms'],v.get('GB_s')) for k,v in l['filter_passes'].items()})"
  f=$(find $O/prof_$ch -name '*kernel_trace.csv' | head -1); rm -f $f
done
echo done
