#!/bin/bash
# Round-2 closing measurement: every GPU test, the three bench lines (c3 default with the CPU
# baseline, c2, c5), rocprofv3 kernel-trace/stats of c3 and c2, PMC FETCH/WRITE traffic passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2f}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; case $rc in 0) ;; *) echo "tests rc=$rc"; exit $rc ;; esac
bash scripts/gpu_r2_bench.sh $T || exit 1
timeout -k 10 400 python3 -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; exit 1; }
cat $O/bench_c5.json | cut -c1-400
