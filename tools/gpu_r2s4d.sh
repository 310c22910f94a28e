# Sum-tree write-back: the top levels' float64 chains folded in one lane (fold levels 0..1,
# default; 0..3: libdq_f3.so) instead of one shuffle round per update: replay / sum-tree /
# rider / north-star tests, then same-box A/B/C vs the previous library (libdq_ref.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s4d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_sumtree.py tests/test_gpu_replay_api.py tests/test_gpu_agent.py tests/test_gpu_northstar.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_f3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_sumtree.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/tests_f3.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 2>/dev/null | tail -1 >> $OUT/bench_f1.log || exit 1
  DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_f3.so timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 2>/dev/null | tail -1 >> $OUT/bench_f3.log || exit 1
  DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_ref.so timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 2>/dev/null | tail -1 >> $OUT/bench_ref.log || exit 1
done
