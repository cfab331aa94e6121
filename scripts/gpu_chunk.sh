#!/bin/bash
# Pass-B pairing + A->B->C chunking experiments: parity tests, then filter-only bench variants.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-chunk}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { echo pytest failed; tail -40 $O/pytest_k.log; exit 1; }
tail -2 $O/pytest_k.log
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
for v in "0 0" "1 0" "1 2" "1 3" "1 4"; do
  set -- $v
  TEXBIAS_KSPACE_PAIR=$1 TEXBIAS_CHUNK_BC=$2 timeout -k 10 300 $B > $O/f_p$1_c$2.json 2> $O/f_p$1_c$2.err || { echo "bench $v failed"; tail -20 $O/f_p$1_c$2.err; exit 1; }
  echo "pair=$1 chunk=$2"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['filter_ms_per_step'], {k:(v['avg_ms'],v.get('GB_s')) for k,v in d['filter_passes'].items()})" $O/f_p$1_c$2.json
done
echo done
