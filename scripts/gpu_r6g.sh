#!/bin/bash
# Compiled 128x64 slab plan for the Gibbs layer: parity + layer-driver bench (eager / graph) + kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6g}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layer_plan.py tests/test_gpu_ops.py tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for g in "" "--graph"; do
  timeout -k 10 300 python3 -u bench.py --model gibbs-layer --steps 20 --warmup 5 $g > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('gibbs-layer $g', d['value'], d['ms_per_step'], {k:(v['kernel'], v['avg_ms'], v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
  TEXBIAS_COMPILED_PLANS=0 timeout -k 10 300 python3 -u bench.py --model gibbs-layer --steps 20 --warmup 5 $g > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('generic gibbs-layer $g', d['value'], d['ms_per_step'], {k:(v['kernel'], v['avg_ms'], v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
done
timeout -k 10 300 python3 -u bench.py --model gibbs-layer --shape 240,240,160 --steps 10 --warmup 3 > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('gibbs-layer 240', d['value'], d['ms_per_step'], {k:(v['kernel'], v['avg_ms'], v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
echo done
