# fused RMSProp (compile-time kind) tests, DQN agent + north-star tests, bench line, config 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_agent.py tests/test_gpu_northstar.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --skip-cpu-baseline > $OUT/bench.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py 400 dqn_pong > $OUT/configs.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/bench_configs.py 300 dqn_pong > $OUT/prof.log 2>&1
