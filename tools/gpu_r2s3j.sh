# IQN: fused tau + cosine draws, mean loss on demand -- IQN tests, config 5 timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_iqn.py tests/test_gpu_agent.py tests/test_gpu_agent_api.py tests/test_gpu_northstar.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_configs.py 150 iqn_breakout > $OUT/iqn.log 2>&1
