# Are the replay riders on the step's critical path?  The bench with the PER set rider,
# the sample rider, or both replaced by empty riders (timing only: stale batches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3o
mkdir -p $OUT
for v in none 0 1 0,1 0,1,2; do
  if [ $v = none ]; then e=""; else e="DQ_EXP_SKIP_RIDERS=$v"; fi
  env $e timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$v -o run -- python3 bench.py --skip-cpu-baseline --skip-configs --steps 300 --gather-iters 20 > $OUT/skip_$v.log 2>&1 || exit 1
  python3 tools/step_timeline_db.py /tmp/prof_$v/run_results.db k_c51 30 > $OUT/timeline_$v.txt 2>&1 || exit 1
  rm -rf /tmp/prof_$v
done
