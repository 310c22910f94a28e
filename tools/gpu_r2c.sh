# rocprof kernel trace of the one-rank RCCL schedule (bench --force-dist)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2c
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/fd -o run -- python3 bench.py --skip-cpu-baseline --steps 300 --force-dist > $OUT/fd.log 2>&1
