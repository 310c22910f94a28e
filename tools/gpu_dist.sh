# The data-parallel path on one GPU: RCCL / multirank tests, the ZeRO-1 two-stream capture
# probe (each variant in its own process), then a same-box A/B of the one-rank RCCL schedule
# (native communicators vs torch collectives) against the no-group bench, and a rocprof
# step timeline of the native one.      gpurun -- bash tools/gpu_dist.sh <out-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
echo "tests rc=$?"; tail -3 $OUT/tests.log
timeout -k 10 300 python -u tools/zero1_capture_probe.py native > $OUT/zero1_native.log 2>&1
echo "zero1 native rc=$?"; tail -2 $OUT/zero1_native.log
timeout -k 10 300 python -u tools/zero1_capture_probe.py torch > $OUT/zero1_torch.log 2>&1
echo "zero1 torch rc=$?"; tail -2 $OUT/zero1_torch.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --steps 2000 > $OUT/b_single_$rep.log 2>&1 || exit 1
  tail -1 $OUT/b_single_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("single", d["value"], d["ms_per_step"])'
  for comm in native torch; do
    timeout -k 10 400 python -u bench.py --skip-cpu-baseline --skip-configs --steps 2000 --force-dist --comm $comm > $OUT/b_${comm}_$rep.log 2>&1 || exit 1
    tail -1 $OUT/b_${comm}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$comm'", d["value"], json.dumps({k: (v["value"], v["comm"]) for k, v in d["schedules"].items()}))'
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --skip-cpu-baseline --skip-configs --force-dist --zero 0 > $OUT/prof.log 2>&1 && \
python3 tools/prof_summary.py /tmp/prof/run_results.db 30 > $OUT/kernel_summary.txt && \
python3 tools/step_timeline_db.py /tmp/prof/run_results.db k_c51 30 > $OUT/step_timeline.txt
