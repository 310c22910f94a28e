# The driver's exact bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5) beside
# 300-step windows of the same build, alternating, in one lease.
#   gpurun -- bash tools/gpu_driver_cmd.sh <out-name> [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-driver_cmd}
mkdir -p $OUT
for rep in $(seq 1 ${2:-2}); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_$rep.log 2>$OUT/driver_$rep.err || exit $?
  echo "[steps 20 warmup 5] $(tail -1 $OUT/driver_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("prime_steps"))')" | tee -a $OUT/windows.log
  timeout -k 10 300 python3 bench.py --steps 300 --skip-cpu-baseline --skip-bf16 --skip-configs > $OUT/s300_$rep.log 2>$OUT/s300_$rep.err || exit $?
  echo "[steps 300 warmup 30] $(tail -1 $OUT/s300_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("prime_steps"))')" | tee -a $OUT/windows.log
done
