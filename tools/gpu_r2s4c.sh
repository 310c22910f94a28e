# Sum-tree write-back: each node's float64 chain folded in one lane by readlane (no shuffle
# rounds): replay / sum-tree / rider / north-star tests, then same-box A/B vs the previous
# library (dopamine_amd/libdq_ref.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s4c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_sumtree.py tests/test_gpu_replay_api.py tests/test_gpu_agent.py tests/test_gpu_northstar.py tests/test_gpu_checkpoint.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 2>/dev/null | tail -1 >> $OUT/bench_new.log || exit 1
  DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_ref.so timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 2>/dev/null | tail -1 >> $OUT/bench_ref.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --skip-cpu-baseline --skip-configs > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/prof/run_results.db k_c51 30 > $OUT/step_timeline.txt
