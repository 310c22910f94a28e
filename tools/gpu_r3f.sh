# The north-star parity tests (mask-pinned Nature CNN), the fc1 tile micro-benchmark, and
# the one-rank RCCL schedule with RCCL's implicit launch order off, same box alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3f
mkdir -p $OUT
timeout -k 10 120 ./tools/micro/fc1_skinny.bin > $OUT/fc1_skinny.log 2>&1; echo "micro rc=$?"; cat $OUT/fc1_skinny.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_northstar.py -m gpu -v -s --timeout 600 --timeout-method thread -k "c51 or rainbow" > $OUT/northstar.log 2>&1
echo "northstar rc=$?"; grep -E "PASSED|FAILED|Error" $OUT/northstar.log | cut -c1-200
grep -o '{"northstar_errors.*' $OUT/northstar.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['northstar_errors'], 'pinned', max(d['grad'].values()), 'unpinned', max(d['grad_unpinned'].values()), 'params', d['params'])"
for rep in 1 2; do
  for cfg in "X=0" "NCCL_LAUNCH_ORDER_IMPLICIT=0"; do
    env $cfg timeout -k 10 300 python -u bench.py --force-dist --zero 0 --skip-cpu-baseline --skip-configs --steps 2000 2>/dev/null | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$cfg'", d["value"])' || exit 1
  done
done
for cfg in "X=0" "NCCL_LAUNCH_ORDER_IMPLICIT=0"; do
  env $cfg timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/q_$cfg -o run -- python3 bench.py --force-dist --zero 0 --skip-cpu-baseline --skip-configs --steps 600 > $OUT/p_$cfg.log 2>&1 || exit 1
  echo "== $cfg"; python3 tools/step_phases.py /tmp/q_$cfg/run_results.db
done
for rep in 1 2; do
  for pr in none main:-1; do
    timeout -k 10 300 python -u tools/iqn_priority.py $pr 150 2>&1 | tail -1 || exit 1
  done
done
