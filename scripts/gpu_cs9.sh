cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "q0 TEXBIAS_CONVMFMA_PERSIST=0" "q1 TEXBIAS_CONVMFMA_PERSIST=1" "q0b TEXBIAS_CONVMFMA_PERSIST=0" "q1b TEXBIAS_CONVMFMA_PERSIST=1"; do set -- $v; t=$1; shift; timeout -k 10 200 env TAG=$t "$@" python3 scripts/diag/conv_kern_bench.py 2>&1 | grep mfma || exit 1; done
bash scripts/gpu_convstep.sh cs9
