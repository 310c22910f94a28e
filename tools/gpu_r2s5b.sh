# IQN: dWe change (unrolled k_colsum) under the float64 / bitwise tests, then a config-5
# rocprof timeline: one median step's kernels and how much of it the GPU is busy
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_iqn.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof5 -o run -- python3 tools/bench_configs.py 150 iqn_breakout > $OUT/prof.log 2>&1 && \
python3 tools/prof_summary.py /tmp/prof5/run_results.db 30 > $OUT/kernel_summary.txt && \
python3 tools/step_timeline_db.py /tmp/prof5/run_results.db k_iqn 30 > $OUT/step_timeline.txt
