# The whole rider chain one launch later (DQ_RIDER_SHIFT=1: write-back in B2, sample in B3,
# gather in B4): rider / chunk / north-star tests under it, then same-box alternating A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s4e
mkdir -p $OUT
DQ_RIDER_SHIFT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_northstar.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  for m in 0 1; do
    DQ_RIDER_SHIFT=$m timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 2>/dev/null | tail -1 >> $OUT/bench_$m.log || exit 1
  done
done
DQ_RIDER_SHIFT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --skip-cpu-baseline --skip-configs > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/prof/run_results.db k_c51 30 > $OUT/step_timeline.txt
