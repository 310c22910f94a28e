# IQN dW1 split-K (compile-time DQ_IQN_SPLIT_W1): 2 (default) vs 1 vs 4, every arm loaded
# through DOPAMINE_AMD_LIB, same box alternating; IQN tests under 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5w
mkdir -p $OUT
DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_w4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_iqn.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for w in 2 1 4; do
    DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_w$w.so timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/w$w.log || exit 1
  done
done
