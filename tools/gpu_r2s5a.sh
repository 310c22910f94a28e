# IQN dWe: 128 x 64 tiles over the E cosine columns, the bias gradient from the dX epilogue
# (DQ_IQN_WE=1, default) vs the 128 x 128 [cos | 1] tile (DQ_IQN_WE=0): tests, same-box A/B, kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_iqn.py tests/test_gpu_agent.py tests/test_gpu_northstar.py tests/test_gpu_agent_api.py -m gpu -v --timeout 240 --timeout-method thread -k "iqn" > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/new.log || exit 1
  DQ_IQN_WE=0 timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/we_wide.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof5 -o run -- python3 tools/bench_configs.py 150 iqn_breakout > $OUT/prof.log 2>&1 && \
python3 tools/prof_summary.py /tmp/prof5/run_results.db 30 > $OUT/kernel_summary.txt
