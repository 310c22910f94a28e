# Where the fc all-reduce starts in the one-rank RCCL schedule: mixed RCCL instances, and
# NCCL graph-mixing / launch-order settings; timelines of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3e
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/p1 -o run -- python3 tools/dist_mixed.py > $OUT/mixed.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/p1/run_results.db k_c51 30 > $OUT/mixed_timeline.txt || exit 1
tail -1 $OUT/mixed.log | cut -c1-120
for cfg in "NCCL_GRAPH_MIXING_SUPPORT=0" "NCCL_LAUNCH_ORDER_IMPLICIT=0"; do
  env $cfg timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/p_$cfg -o run -- python3 bench.py --force-dist --zero 0 --skip-cpu-baseline --skip-configs > $OUT/b_$cfg.log 2>&1 && \
  python3 tools/step_timeline_db.py /tmp/p_$cfg/run_results.db k_c51 30 > $OUT/timeline_$cfg.txt || exit 1
  tail -1 $OUT/b_$cfg.log | cut -c1-120
done
for rep in 1 2; do
  timeout -k 10 300 python -u tools/dist_mixed.py --steps 2000 2>/dev/null | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("mixed", d["value"])' || exit 1
  timeout -k 10 300 python -u bench.py --force-dist --zero 0 --skip-cpu-baseline --skip-configs --steps 2000 2>/dev/null | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("native", d["value"])' || exit 1
done
