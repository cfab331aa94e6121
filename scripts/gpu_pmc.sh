#!/bin/bash
# PMC counters of the filter chain kernels (pass_bench C3, no flush), one counter group per
# pass, plus the list of counters.  Usage (GPU box): bash scripts/gpu_pmc.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3m}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- python3 scripts/pass_bench.py --config c3 --iters 5 --warmup 2 --flush-mb 0 > $O/pmc$i.out 2> $O/pmc$i.err || { echo "pmc $i failed"; tail -3 $O/pmc$i.err; }
done

echo done
