#!/bin/bash
# Round-6 first look: access-order microbenchmark, S&P sweep kernel parity + timing, event-fence A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6a}; mkdir -p $O
timeout -k 10 180 ./scripts/micro/order_bw 10 > $O/order.jsonl 2> $O/order.err || { echo order failed; tail -5 $O/order.err; exit 1; }
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_dropin.py tests/test_gpu_fusedchain.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in sweep geom; do
  for f in 0 1; do
    TEXBIAS_SAP=$v TEXBIAS_EVENT_FENCE=$f timeout -k 10 120 python3 -u scripts/pass_bench.py --tag sap_${v}_fence$f >> $O/pass.jsonl 2>> $O/pass.err || { echo pass failed; tail -5 $O/pass.err; exit 1; }
  done
done
cat $O/pass.jsonl | cut -c1-400
for v in sweep geom; do
  TEXBIAS_SAP=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo bench failed; tail -5 $O/bench_$v.err; exit 1; }
  cut -c1-300 $O/bench_$v.json
  python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print({k:(v['avg_ms'],v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['filter_ms_per_step'], d['roofline']['frac'])"
done
echo done
