# Config 5 (IQN; CFG=dqn_pong: config 2) steps/s alternating in-tree / the given builds, 2 rounds.
#   gpurun -- bash tools/gpu_iqn_bench_ab.sh <out-name> ab/X/libdopamine_amd.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-iqn_bench_ab}
shift
mkdir -p $OUT
for rep in 1 2; do
  for lib in "" "$@"; do
    line=$(DOPAMINE_AMD_LIB=$lib timeout -k 10 200 python tools/bench_configs.py ${STEPS:-300} ${CFG:-iqn_breakout} 2>>$OUT/err.log | tail -1) || exit 1
    echo "[${lib:-in-tree}] $line" | tee -a $OUT/ab.log
  done
done
