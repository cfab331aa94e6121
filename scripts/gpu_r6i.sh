#!/bin/bash
# U-Net level hand-offs: bitwise test, train-step tests, bench C3, remaining small ops.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6i}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_unet_pack.py tests/test_gpu_train_prod.py tests/test_gpu_ddp.py tests/test_gpu_norm.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('c3', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
timeout -k 10 300 python3 -u scripts/diag/step_small_ops.py > $O/small_ops.txt 2> $O/small_ops.err || { echo ops failed; tail -3 $O/small_ops.err; exit 1; }
head -30 $O/small_ops.txt | cut -c1-200
echo done
