#!/bin/bash
# Round 3: where the first (warmup) train step spends its time, and the f64-anchored whole-step test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3c}; mkdir -p $O
export TEXBIAS_MIOPEN_DIR=$GRAFT_REPO_ROOT/gpurun_out/miopen
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-cudnn-benchmark > $O/nobench.json 2> $O/nobench.err || { echo nobench failed; tail -5 $O/nobench.err; exit 1; }
grep "warmup step" $O/nobench.err; cut -c1-160 $O/nobench.json
MIOPEN_FIND_MODE=FAST timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/fast.json 2> $O/fast.err || { echo fast failed; tail -5 $O/fast.err; exit 1; }
grep "warmup step" $O/fast.err; cut -c1-160 $O/fast.json
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 560 --timeout-method thread tests/test_gpu_train_prod.py -k matches_aten > $O/whole.log 2>&1; rc=$?
grep -E "loss texbias|  model|passed|failed|Error" $O/whole.log | head -20
echo rc=$rc
