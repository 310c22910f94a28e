# k_c51 stage stamps; rocprof kernel traces of the bench with and without replay riders
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2b
mkdir -p $OUT
DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_c51prof.so timeout -k 10 120 python -u tools/c51_stamps.py > $OUT/c51_stamps.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ride1 -o run -- python3 bench.py --skip-cpu-baseline --steps 300 > $OUT/ride1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ride0 -o run -- python3 bench.py --skip-cpu-baseline --steps 300 --ride 0 > $OUT/ride0.log 2>&1
