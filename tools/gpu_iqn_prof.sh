# rocprofv3 kernel summaries of config 5 (IQN): the two-stream step and the serial one.
#   gpurun -- bash tools/gpu_iqn_prof.sh <out-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-iqn_prof}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p2 -o run -- python3 tools/bench_configs.py 150 iqn_breakout > $OUT/prof2.log 2>&1 && \
python3 tools/prof_summary.py /tmp/p2/run_results.db 25 > $OUT/two_stream_kernels.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p1 -o run -- python3 tools/bench_configs.py 150 iqn_breakout pipeline=0 > $OUT/prof1.log 2>&1 && \
python3 tools/prof_summary.py /tmp/p1/run_results.db 25 > $OUT/serial_kernels.txt && \
python3 tools/step_timeline_db.py /tmp/p1/run_results.db k_iqn 30 > $OUT/serial_timeline.txt
