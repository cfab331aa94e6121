#!/bin/bash
# Stage attribution of passes A' and C' (TEXBIAS_BAND_DIAG masks; results invalid by design) + C2 line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6b}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unet_pack.py tests/test_gpu_chain_glue.py tests/test_gpu_conv.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for d in 0 0x1 0x2 0x4 0x8 0xc 0x400 0x800 0xc00 0x1000 0x1400 0x1c00 0x2000; do
  TEXBIAS_BAND_DIAG=$((d)) timeout -k 10 120 python3 -u scripts/pass_bench.py --tag diag_$d >> $O/diag.jsonl 2>> $O/diag.err || { echo diag $d failed; tail -5 $O/diag.err; exit 1; }
done
python3 - <<PY
import json
for l in open("$O/diag.jsonl"):
    d = json.loads(l)
    print(d["tag"], {k: d[k]["us"] for k in ("forward", "kspace", "inverse", "salt_pepper") if k in d})
PY
timeout -k 10 120 python3 -u scripts/pass_bench.py --config c2 --tag c2 >> $O/c2.jsonl 2>> $O/c2.err || { echo c2 failed; exit 1; }
cat $O/c2.jsonl
echo done
