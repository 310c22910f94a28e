# In-step cost of the gather rider: rocprof kernel traces of the bench as is and with the
# gather rider replaced by an empty one (DQ_EXP_SKIP_GATHER=1: same launches, no gather blocks)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3i
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/ride1 -o run -- python3 bench.py --skip-cpu-baseline --skip-configs --steps 300 > $OUT/ride1.log 2>&1 && \
DQ_EXP_SKIP_GATHER=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/skip -o run -- python3 bench.py --skip-cpu-baseline --skip-configs --steps 300 > $OUT/skip.log 2>&1
