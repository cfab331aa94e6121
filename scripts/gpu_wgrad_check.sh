#!/bin/bash
# wgrad change: conv / train-step parity at the bench shapes, then the C3 bench with a kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-wg}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_train_prod.py > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -4 gpurun_out/$T/tests.log; case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/trace -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo bench failed; tail -3 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json | cut -c1-300
python3 - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/$T/trace/run_kernel_stats.csv")):
    if "wgrad" in r["Name"]: print(f'{float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]:>4}  {r["Name"][:80]}')
PY
