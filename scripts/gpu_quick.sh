#!/bin/bash
# conv/loss parity tests, wgrad microbench, bench line, steady-state kernel profile
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_loss.py tests/test_gpu_norm.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo tests failed; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('vols/s',d['value'],'ms/step',d['ms_per_step'],'filter',d['filter_passes'])"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > $O/prof_bench.json 2> $O/prof_bench.err || { echo prof failed; tail -30 $O/prof_bench.err; exit 1; }
python3 scripts/steady_stats.py $O/prof/run_kernel_trace.csv --steps 5 --top 24 > $O/steady.txt 2>&1; head -28 $O/steady.txt | cut -c1-120
echo done
