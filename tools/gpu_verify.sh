# Verification at HEAD on one GPU: every GPU test, smoke, the default bench line, and a
# rocprofv3 kernel-trace summary + step timeline of the bench.
#   gpurun -- bash tools/gpu_verify.sh <out-name> [tests|notests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-verify}
mkdir -p $OUT
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"
  tail -3 $OUT/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --skip-cpu-baseline --skip-bf16 > $OUT/prof.log 2>&1 && \
python3 tools/prof_summary.py /tmp/prof/run_results.db 30 > $OUT/kernel_summary.txt && \
python3 tools/step_timeline_db.py /tmp/prof/run_results.db k_c51 30 > $OUT/step_timeline.txt && \
python3 tools/gather_launches.py /tmp/prof/run_results.db 400 32 $OUT/prof.log > $OUT/gather_launches.txt
