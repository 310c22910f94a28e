# device epsilon-greedy: agent tests, then the acting-loop benchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3m
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_agent_api.py tests/test_gpu_runner.py tests/test_gpu_cartpole.py tests/test_gpu_northstar.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/bench_actor.py 2000 > $OUT/actor.log 2>&1
