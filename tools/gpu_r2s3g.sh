# ZeRO-1: multirank (gloo, two ranks on one GPU) and one-rank RCCL tests, then the
# one-rank RCCL schedule with and without the sharded fc update
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py -m gpu -v --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --force-dist --steps 400 --gather-iters 20 > $OUT/fd.log 2>&1 && \
timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --force-dist --zero 1 --steps 400 --gather-iters 20 > $OUT/fd_zero.log 2>&1
