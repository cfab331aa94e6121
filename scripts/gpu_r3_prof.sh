#!/bin/bash
# Round 3: rocprofv3 kernel trace of the filter chain (pass_bench, with and without the cache flush),
# then the listed GPU tests.  Usage (GPU box): bash scripts/gpu_r3_prof.sh TAG [tests...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r3p}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 200 --timeout-method thread -m gpu tests/test_gpu_band.py > $O/tests_band.log 2>&1
rc=$?; grep -cE "PASSED" $O/tests_band.log; [ $rc = 0 ] || { grep -E "Error|assert" $O/tests_band.log | head -30 | cut -c1-300; exit $rc; }
for fl in 1024 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_f$fl -o run -- python3 scripts/pass_bench.py --config c3 --iters 20 --flush-mb $fl > $O/prof_c3_f$fl.out 2> $O/prof_c3_f$fl.err || { echo prof $fl failed; tail -5 $O/prof_c3_f$fl.err; exit 1; }
  f=$(find $O/prof_c3_f$fl -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('flush $fl', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --tb=short --timeout 600 --timeout-method thread -m gpu "$@" > $O/tests_extra.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|loss texbias|^  model" $O/tests_extra.log | tail -60; [ $rc = 0 ] || { tail -30 $O/tests_extra.log | cut -c1-300; exit $rc; }
fi
echo done
