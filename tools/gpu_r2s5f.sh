# Control for the library A/Bs: both arms loaded through DOPAMINE_AMD_LIB (new = epilogue
# loads together, prev = before it), plus the default path (= new) as an A/A arm
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5f
mkdir -p $OUT
for i in 1 2 3; do
  DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdopamine_amd_prev.so timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/prev_env.log || exit 1
  DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdopamine_amd_new.so timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/new_env.log || exit 1
  timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/new_default.log || exit 1
done
