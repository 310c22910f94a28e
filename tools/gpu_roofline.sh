# Per-launch roofline of the Rainbow step: a kernel trace, then FETCH_SIZE and WRITE_SIZE in
# passes of their own (rocprofv3 --pmc, one counter block each; eager launches of the same
# kernels, --no-graph), then the table.
#   gpurun -- bash tools/gpu_roofline.sh <out-name> [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-roofline}
shift
mkdir -p $OUT
ARGS="--skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 $*"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rt -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d /tmp/rf -o run --output-format csv -- python3 bench.py $ARGS --steps 120 --no-graph > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d /tmp/rw -o run --output-format csv -- python3 bench.py $ARGS --steps 120 --no-graph > $OUT/write.log 2>&1 || exit 1
python3 tools/launch_roofline.py /tmp/rt/run_results.db /tmp/rf /tmp/rw > $OUT/launch_roofline.md && cat $OUT/launch_roofline.md
python3 tools/step_timeline_db.py /tmp/rt/run_results.db k_c51 30 > $OUT/step_timeline.txt
