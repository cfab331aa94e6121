#!/bin/bash
# Round-2 GPU check of the newer rows: preprocessing + DCGAN tests, then the c5 bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2n}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prep.py tests/test_gpu_dcgan.py > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -12 gpurun_out/$T/tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/$T/bench_c5.json 2> gpurun_out/$T/bench_c5.err || { echo bench c5 failed; tail -5 gpurun_out/$T/bench_c5.err; exit 1; }
cat gpurun_out/$T/bench_c5.json
