#!/bin/bash
# Pass C' one-round-trip key reduction: parity tests touching the keys, then the C3 bench twice and C2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6j}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_kernels.py tests/test_gpu_fusedchain.py tests/test_gpu_c4_extremes.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('c3', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['filter_passes'].items()}, d['roofline']['kernel'], d['roofline']['frac'])"
done
timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('c2', d['value'], {k:v['avg_ms'] for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
echo done
