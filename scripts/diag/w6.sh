set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/w6; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py -m gpu > $O/conv.log 2>&1; grep -E "PASSED|FAILED|Error|assert" $O/conv.log | tail -25
timeout -k 10 300 python -u scripts/wgrad_bench.py > $O/wgrad.txt 2>&1; cat $O/wgrad.txt
TEXBIAS_WGRAD_ZM=0 timeout -k 10 300 python -u scripts/wgrad_bench.py > $O/wgrad_old.txt 2>&1; head -7 $O/wgrad_old.txt
timeout -k 10 400 python -u scripts/diag/adn_check.py > $O/adn.txt 2>&1; grep -v Warn $O/adn.txt | tail -12
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train_prod.py -m gpu -s -k matches_aten > $O/train_prod.log 2>&1; grep -E "passed|failed|loss texbias|texbias .* aten-f32" $O/train_prod.log | head -12
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; cut -c1-300 $O/bench.json
echo done
