cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "r3 TEXBIAS_CONV16_RING=3" "r4 TEXBIAS_CONV16_RING=4" "r3pf TEXBIAS_CONV16_RING=3 TEXBIAS_CONV16_PF=1" "r4pf TEXBIAS_CONV16_PF=1" "r3b TEXBIAS_CONV16_RING=3" "r4b TEXBIAS_CONV16_RING=4"; do set -- $v; t=$1; shift; timeout -k 10 200 env TAG=$t "$@" python3 scripts/diag/conv_kern_bench.py 2>&1 | grep fwd16 || exit 1; done
bash scripts/gpu_convstep.sh cs2
