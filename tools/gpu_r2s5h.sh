# Re-measure the C51 loss split (target half beside the online fused head, --split-c51 1)
# against the one-kernel loss at HEAD (the schedule has changed since round 2's 7,218 vs 7,290)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5h
mkdir -p $OUT
for i in 1 2 3; do
  for m in 0 1; do
    timeout -k 10 200 python -u bench.py --skip-cpu-baseline --skip-configs --steps 3000 --split-c51 $m 2>/dev/null | tail -1 >> $OUT/split_$m.log || exit 1
  done
done
