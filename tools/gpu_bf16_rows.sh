# The bf16 throughput row (NOT fp32 parity): Rainbow bench alternating in-tree / the bf16
# build, and config 5 (IQN) on both.   gpurun -- bash tools/gpu_bf16_rows.sh <out> <lib>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-bf16_rows}
mkdir -p $OUT
bash tools/ab_lib.sh $2 | tee $OUT/rainbow_ab.log
for lib in "" $2; do
  line=$(DOPAMINE_AMD_LIB=$lib timeout -k 10 200 python tools/bench_configs.py 300 iqn_breakout 2>>$OUT/err.log | tail -1) || exit 1
  echo "[${lib:-in-tree}] $line" | tee -a $OUT/iqn.log
done
