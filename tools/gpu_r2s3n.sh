# asynchronous staged add + device max priority + device epsilon-greedy: replay / agent /
# checkpoint / runner tests, then the acting-loop benchmark and its phase breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread --deselect tests/test_gpu_cartpole.py::test_cartpole_dqn_steps_match_float64_oracle > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_cartpole.py -v --timeout 240 --timeout-method thread > $OUT/tests_cartpole.log 2>&1
timeout -k 10 400 python -u tools/bench_actor.py 2000 > $OUT/actor.log 2>&1 && \
timeout -k 10 400 python -u tools/actor_phases.py > $OUT/phases.log 2>&1
