# IQN config 5: pipelined (target forward on the prefetch stream) vs one stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3f
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_configs.py 150 iqn_breakout > $OUT/pipe.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py 150 iqn_breakout pipeline=0 > $OUT/nopipe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 tools/bench_configs.py 120 iqn_breakout pipeline=0 > $OUT/prof.log 2>&1
