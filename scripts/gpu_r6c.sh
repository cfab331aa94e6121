#!/bin/bash
# Split-f16 pass A': parity (band / chain / extremes / drop-in tests), A/B timing vs the f32 D product.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6c}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_kernels.py tests/test_gpu_fusedchain.py tests/test_gpu_c4_extremes.py tests/test_gpu_dropin.py tests/test_gpu_half.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for f in 1 0 1 0; do
  TEXBIAS_BAND_FWD16=$f timeout -k 10 120 python3 -u scripts/pass_bench.py --tag fwd16_$f >> $O/pass.jsonl 2>> $O/pass.err || { echo pass failed; tail -5 $O/pass.err; exit 1; }
  TEXBIAS_BAND_FWD16=$f timeout -k 10 120 python3 -u scripts/pass_bench.py --config c2 --tag c2_fwd16_$f >> $O/pass.jsonl 2>> $O/pass.err || { echo pass failed; tail -5 $O/pass.err; exit 1; }
done
python3 - <<PY
import json
for l in open("$O/pass.jsonl"):
    d = json.loads(l)
    print(d["tag"], {k: d[k]["us"] for k in ("forward", "kspace", "inverse", "salt_pepper") if k in d})
PY
for f in 1 0; do
  TEXBIAS_BAND_FWD16=$f timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$f.json 2> $O/bench_$f.err || { echo bench failed; tail -5 $O/bench_$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$f.json')); print('$f', d['value'], {k:(v['avg_ms'],v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['filter_ms_per_step'], d['roofline']['frac'])"
done
echo done
