# Serial (one-stream) IQN kernel summaries per library: in-tree, then each given build.
#   gpurun -- bash tools/gpu_iqn_serial_ab.sh <out-name> ab/X/libdopamine_amd.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-iqn_serial_ab}
shift
mkdir -p $OUT
for lib in "" "$@"; do
  n=$(basename $(dirname ${lib:-x/in-tree/x}))
  DOPAMINE_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/s_$n -o run -- python3 tools/bench_configs.py 150 iqn_breakout pipeline=0 > $OUT/prof_$n.log 2>&1 || exit 1
  python3 tools/prof_summary.py /tmp/s_$n/run_results.db 12 > $OUT/serial_$n.txt
  echo "== $n"; head -10 $OUT/serial_$n.txt | cut -c1-150
done
