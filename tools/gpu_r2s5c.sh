# IQN: one stream (pipeline=0: the target forward before the online one, nothing
# overlapped) vs the two-stream schedule (target forward beside the online backward),
# same box alternating; then the one-stream timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5c
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/two_stream.log || exit 1
  timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout pipeline=0 2>&1 | tail -1 >> $OUT/one_stream.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof5 -o run -- python3 tools/bench_configs.py 150 iqn_breakout pipeline=0 > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/prof5/run_results.db k_iqn 30 > $OUT/step_timeline.txt
