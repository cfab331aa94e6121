#!/bin/bash
# Split-f16 pass A' A/B (pass timing, C3 and C2), occupancy print, quick band parity.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6d}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_kernels.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TEXBIAS_BAND_VERBOSE=1 timeout -k 10 120 python3 -u scripts/pass_bench.py --iters 3 --tag verbose > /dev/null 2> $O/verbose.err || { echo verbose failed; tail -5 $O/verbose.err; exit 1; }
grep texbias $O/verbose.err | sort | uniq
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
echo done
