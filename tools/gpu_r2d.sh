# configs 2 (DQN/Pong) and 5 (IQN/Breakout): bench_configs lines + rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2d
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_configs.py 300 > $OUT/configs.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dqn -o run -- python3 tools/bench_configs.py 300 dqn_pong > $OUT/dqn_prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/iqn -o run -- python3 tools/bench_configs.py 150 iqn_breakout > $OUT/iqn_prof.log 2>&1
