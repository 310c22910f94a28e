# one-rank RCCL schedule after the capture-order change: tests, bench line, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --skip-cpu-baseline --steps 400 --gather-iters 20 --force-dist > $OUT/fd.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/fdp -o run -- python3 bench.py --skip-cpu-baseline --steps 300 --gather-iters 20 --force-dist > $OUT/fdp.log 2>&1
