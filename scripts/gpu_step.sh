#!/bin/bash
# Train-step measurement: the C3 bench line (no CPU baseline) and the steady-state kernel breakdown of
# the same command under rocprofv3 --kernel-trace --stats.  Usage (GPU box): TAG [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-step}; shift
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $O/prof.json 2> $O/prof.err || { echo prof failed; tail -5 $O/prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/steady_stats.py $f --steps 20 --marker k_band_fwd --top 60 --calls "${CALLS:-.}" > $O/steady.txt && head -30 $O/steady.txt
rm -f $f
cp $(find $O/prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
echo done
