#!/bin/bash
# Bench C3 three times (the driver's command), C2 line with its CPU baseline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6e}; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || { echo bench failed; tail -5 $O/bench_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$i.json')); print('$i', d['value'], {k:(v['avg_ms'],v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['filter_ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
timeout -k 10 600 python3 -u bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err || { echo c2 failed; tail -5 $O/bench_c2.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/bench_c2.json')); print('c2', d['value'], {k:(v['avg_ms'],v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['roofline']['kernel'], d['roofline']['frac'], d.get('cpu_baseline', {}).get('value'))"
echo done
