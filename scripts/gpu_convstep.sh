#!/bin/bash
# Conv kernel change check: the conv GPU tests, then the C3 step line + steady breakdown.  Usage: TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-cs}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_up.py tests/test_gpu_conv_gemm.py tests/test_gpu_conv.py tests/test_gpu_norm.py tests/test_gpu_loss.py tests/test_gpu_train_prod.py tests/test_gpu_ddp.py tests/test_gpu_ops.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpu_step.sh $T/step || exit 1
