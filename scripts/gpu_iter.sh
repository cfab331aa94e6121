#!/bin/bash
# Development iteration on the GPU box: the train-step GPU tests, then the C3 bench line and its
# steady-state kernel breakdown (scripts/gpu_step.sh).  Usage: TAG [test files...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-iter}; shift
O=gpurun_out/$T; mkdir -p $O
TESTS=${@:-tests/test_gpu_norm.py tests/test_gpu_conv_gemm.py tests/test_gpu_conv.py tests/test_gpu_conv_up.py tests/test_gpu_ops.py tests/test_gpu_ddp.py tests/test_gpu_train_prod.py}
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpu_step.sh $T
