# The data-parallel path on one GPU at HEAD: RCCL / multirank tests, then a same-box A/B of
# the one-rank RCCL schedule (both data-parallel schedules, native communicators) against the
# no-group bench, and a rocprof step timeline of the all-reduce schedule.
#   gpurun -- bash tools/gpu_dist_bench.sh <out-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist_bench}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --steps 2000 > $OUT/b_single_$rep.log 2>&1 || exit 1
  tail -1 $OUT/b_single_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("single", d["value"], d["ms_per_step"])'
  timeout -k 10 400 python -u bench.py --skip-cpu-baseline --skip-configs --steps 2000 --force-dist > $OUT/b_dist_$rep.log 2>&1 || exit 1
  tail -1 $OUT/b_dist_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("force-dist", d["value"], json.dumps({k: (v["value"], v["per_rank_ms_per_step"], v["comm"]) for k, v in d["schedules"].items()}))'
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --skip-cpu-baseline --skip-configs --force-dist --zero 0 > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/prof/run_results.db k_c51 30 > $OUT/step_timeline.txt
