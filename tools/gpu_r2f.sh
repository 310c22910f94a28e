# A/B of the split C51 loss (head_from 8) vs the one-kernel loss (head_from 6): bench lines
# and rocprof kernel traces of each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2f
mkdir -p $OUT
for v in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --skip-cpu-baseline --steps 600 --gather-iters 20 --split-c51 $v > $OUT/b$v.log 2>&1 || exit $?
  echo "split=$v $(tail -1 $OUT/b$v.log | cut -c1-120)"
done
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p$v -o run -- python3 bench.py --skip-cpu-baseline --steps 300 --gather-iters 20 --split-c51 $v > $OUT/p$v.log 2>&1 || exit $?
done
