#!/bin/bash
# GPU check of the compiled-plan slab passes and the DMA-staged weight gradient: parity tests,
# full bench line, filter-only bench at both workgroup sizes, rocprofv3 kernel-trace summary.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ct}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for nt in 768 512; do
  TEXBIAS_CT_NT=$nt timeout -k 10 300 python bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline > $O/filter_nt$nt.json 2> $O/filter_nt$nt.err || { echo "filter bench nt=$nt failed"; tail -20 $O/filter_nt$nt.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/filter_nt$nt.json').read().strip().splitlines()[-1]);print('nt=$nt', d['filter_passes'])"
done
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > $O/prof_bench.json 2> $O/prof_bench.err || { echo prof failed; tail -30 $O/prof_bench.err; exit 1; }
echo done
