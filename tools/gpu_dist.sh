# N > 1 checks on one GPU: the HIP event-query-under-capture micro, the RCCL and
# multi-rank tests (world 2, checkpoint resume), then the world-8 test.
#   gpurun -- bash tools/gpu_dist.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist}
mkdir -p $OUT
if [ -z "$DQ_DIST_NOTESTS" ]; then
# the HIP event-query-under-capture micro, built here if missing
[ -x tools/micro/event_query_capture.bin ] || hipcc --offload-arch=gfx950 -O2 -o tools/micro/event_query_capture.bin tools/micro/event_query_capture.hip
timeout -k 10 60 tools/micro/event_query_capture.bin > $OUT/evq.log 2>&1; echo "evq rc=$?"; cat $OUT/evq.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py tests/test_gpu_peer.py "tests/test_gpu_agent.py::test_fused_optimizer_without_gradient_stores_is_bitwise_the_same" -m gpu -v -s --timeout 600 --timeout-method thread -k "not world8" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v -s --timeout 850 --timeout-method thread -k world8 > $OUT/world8.log 2>&1
echo "world8 rc=$?"; tail -5 $OUT/world8.log
fi
# DQ_DIST_MODEL=1: also the one-rank RCCL schedule (bench --force-dist, every collective
# executed) beside the no-group bench, its rocprof step timeline and the N = 8 model from it
if [ -n "$DQ_DIST_MODEL" ]; then
  for rep in 1 2; do
    for extra in "" "--force-dist --schedules peer" "--force-dist --schedules allreduce" "--force-dist --schedules zero1"; do
      line=$(timeout -k 10 240 python bench.py --steps 2000 --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 $extra 2>>$OUT/err.log | tail -1) || exit 1
      echo "[${extra:-no group}] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT/one_rank_ab.log
    done
  done
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rd -o run -- python3 bench.py --force-dist --schedules ${DQ_DIST_SCHEDULE:-peer} --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 > $OUT/prof_dist.log 2>&1 || exit 1
  python3 tools/step_timeline_db.py /tmp/rd/run_results.db k_c51 30 > $OUT/dist_step_timeline.txt
  # the no-group step: DQ_SINGLE_TL = a step timeline of the same build (gpu_verify.sh's)
  single=$(python3 -c "import re; print(re.search(r'median step ([0-9.]+)', open('$DQ_SINGLE_TL').read()).group(1))" 2>/dev/null || echo 122.5)
  python3 tools/n8_model.py $OUT/dist_step_timeline.txt $single > $OUT/n8_model.txt; cat $OUT/n8_model.txt
fi
