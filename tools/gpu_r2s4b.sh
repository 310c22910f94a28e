# PER write-back + next draw chained in one rider block (DQ_SET_SAMPLE=1: gather stays in
# launch 3; =2: gather in launch 2): the rider / chunk / north-star tests under each, then a
# same-box alternating bench A/B against the separate riders (0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s4b
mkdir -p $OUT
for m in 1 2; do
  DQ_SET_SAMPLE=$m timeout -k 10 400 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_northstar.py -m gpu -v --timeout 240 --timeout-method thread -k "rainbow or riders or fused or chunks or eager" > $OUT/tests_$m.log 2>&1
  rc=$?
  echo "pytest mode $m rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for i in 1 2 3; do
  for m in 0 1 2; do
    DQ_SET_SAMPLE=$m timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 2>/dev/null | tail -1 >> $OUT/bench_$m.log || exit 1
  done
done
