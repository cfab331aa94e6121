#!/bin/bash
# Round 3: MIOpen find-db / kernel cache persistence -- bench.py twice with the cache under
# gpurun_out/miopen (the first run fills it, the second reuses it).  Usage: bash scripts/gpu_r3_miopen.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3b}
mkdir -p $O gpurun_out/miopen
export TEXBIAS_MIOPEN_DIR=$GRAFT_REPO_ROOT/gpurun_out/miopen
for run in 1 2; do
  timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$run.json 2> $O/bench_$run.err || { echo "bench $run failed"; tail -5 $O/bench_$run.err; exit 1; }
  grep "warmup step" $O/bench_$run.err; cut -c1-200 $O/bench_$run.json
done
du -sh gpurun_out/miopen; find gpurun_out/miopen -type f | head -20
echo done
