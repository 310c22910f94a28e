# fused RMSProp test + the Rainbow bench line (codegen check after the optimizer-kind change)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn.py -m gpu -v --timeout 240 --timeout-method thread -k "rmsprop or dqn_loss" > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --skip-cpu-baseline > $OUT/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --skip-cpu-baseline > $OUT/bench2.log 2>&1
