#!/bin/bash
# Small-change check: the given GPU tests, C3 step line + steady breakdown, and the default-chain
# filter-only line with the S&P block order reversed vs not.  Usage: TAG TESTS...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-misc}; shift
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread "$@" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rv in 0; do
  timeout -k 10 200 env TEXBIAS_SAP_REV=$rv python3 -u bench.py --filter-only --steps 30 --warmup 5 --no-cpu-baseline > $O/f$rv.json 2> $O/f$rv.err || { echo "filter $rv failed"; tail -5 $O/f$rv.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/f$rv.json').read().strip().splitlines()[-1]); print('rev $rv', d['filter_ms_per_step'], {k: (v['kernel'], v['avg_ms']) for k, v in d['filter_passes'].items()})"
done
bash scripts/gpu_step.sh $T/step || exit 1
