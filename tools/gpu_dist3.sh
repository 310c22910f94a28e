# N > 1 schedule on one GPU (one-rank RCCL, all-reduce schedule): HIP graph runtime settings
# that change how cross-queue edges are dispatched, same box alternating; then the
# capture-fork repro at 1 and 2 steps (a segfault ends the script: it runs last).
#   gpurun -- bash tools/gpu_dist3.sh <out-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist3}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "X=0" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=4" "GPU_MAX_HW_QUEUES=8"; do
    env $cfg timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --steps 2000 --force-dist --zero 0 > $OUT/b_${cfg}_$rep.log 2>&1 || exit 1
    tail -1 $OUT/b_${cfg}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'"$cfg"'", d["value"], d["ms_per_step"])'
  done
done
env DEBUG_HIP_GRAPH_BATCH_SIZE=1 timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof -o run -- python3 bench.py --skip-cpu-baseline --skip-configs --force-dist --zero 0 > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/prof/run_results.db k_c51 30 > $OUT/step_timeline_batch1.txt || exit 1
timeout -k 10 120 python -u tools/capture_fork_repro.py 1 plain > $OUT/repro_1_plain.log 2>&1 || { echo "repro 1 plain rc=$?"; exit 1; }
tail -1 $OUT/repro_1_plain.log
timeout -k 10 120 python -u tools/capture_fork_repro.py 2 plain > $OUT/repro_2_plain.log 2>&1
echo "repro 2 plain rc=$?"; tail -1 $OUT/repro_2_plain.log
