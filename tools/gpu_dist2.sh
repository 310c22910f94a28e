# N > 1 schedule experiments on one GPU (one-rank RCCL): fc branch captured after (default)
# or before the backward tail, same box alternating, + rocprof step timeline of each; then
# the capture-fork repro (tools/capture_fork_repro.py), the expected crash last.
#   gpurun -- bash tools/gpu_dist2.sh <out-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist2}
mkdir -p $OUT
for rep in 1 2; do
  for v in "" "--branch-first"; do
    timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --steps 2000 --force-dist --zero 0 $v > $OUT/b${v}_$rep.log 2>&1 || exit 1
    tail -1 $OUT/b${v}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'"${v:-default}"'", d["value"], d["ms_per_step"])'
  done
done
for v in "" "--branch-first"; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof$v -o run -- python3 bench.py --skip-cpu-baseline --skip-configs --force-dist --zero 0 $v > $OUT/prof$v.log 2>&1 || exit 1
  python3 tools/step_timeline_db.py /tmp/prof$v/run_results.db k_c51 30 > $OUT/step_timeline$v.txt || exit 1
done
timeout -k 10 120 python -u tools/capture_fork_repro.py 4 direct > $OUT/repro_4_direct.log 2>&1 || { echo "repro 4 direct rc=$?"; exit 1; }
tail -1 $OUT/repro_4_direct.log
timeout -k 10 120 python -u tools/capture_fork_repro.py 1 plain > $OUT/repro_1_plain.log 2>&1 || { echo "repro 1 plain rc=$?"; exit 1; }
tail -1 $OUT/repro_1_plain.log
timeout -k 10 120 python -u tools/capture_fork_repro.py 4 plain > $OUT/repro_4_plain.log 2>&1
echo "repro 4 plain rc=$?"; tail -1 $OUT/repro_4_plain.log
