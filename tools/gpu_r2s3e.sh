# IQN config-5 kernel trace for the step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3e
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 tools/bench_configs.py 120 iqn_breakout > $OUT/prof.log 2>&1
