# N > 1 checks on one GPU: the HIP event-query-under-capture micro, the RCCL and
# multi-rank tests (world 2, checkpoint resume), then the world-8 test.
#   gpurun -- bash tools/gpu_dist.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist}
mkdir -p $OUT
timeout -k 10 60 tools/micro/event_query_capture.bin > $OUT/evq.log 2>&1; echo "evq rc=$?"; cat $OUT/evq.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py "tests/test_gpu_agent.py::test_fused_optimizer_without_gradient_stores_is_bitwise_the_same" -m gpu -v -s --timeout 600 --timeout-method thread -k "not world8" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v -s --timeout 850 --timeout-method thread -k world8 > $OUT/world8.log 2>&1
echo "world8 rc=$?"; tail -5 $OUT/world8.log
