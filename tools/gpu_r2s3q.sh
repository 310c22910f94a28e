# ZeRO-1 captured: RCCL + multirank tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py -m gpu -v --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
