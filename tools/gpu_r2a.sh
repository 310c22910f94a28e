# GPU verification run: all GPU tests (no -x: a failing assertion does not stop the
# rest), smoke, bench, a rocprofv3 kernel-trace summary of the bench, then the
# CartPole parity test on its own (last: it exercises torch autograd graph capture).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${DQ_TAG:-r2a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread --deselect tests/test_gpu_cartpole.py::test_cartpole_dqn_steps_match_float64_oracle > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --skip-cpu-baseline > $OUT/prof.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_cartpole.py -v --timeout 240 --timeout-method thread > $OUT/gpu_tests_cartpole.log 2>&1
