# IQN FC1 split-K (DQ_IQN_SPLIT_FC1): 4 (default: 512 / 768 blocks online / target on 512
# two-block slots) vs 8 (1024 / 1536: whole rounds) vs 6; tests under 8, same-box alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5g
mkdir -p $OUT
DQ_IQN_SPLIT_FC1=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_iqn.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for s in 4 8 6; do
    DQ_IQN_SPLIT_FC1=$s timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/split_$s.log || exit 1
  done
done
