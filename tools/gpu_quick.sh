# Quick GPU check: chosen test files, then the bench line.   DQ_TESTS="tests/a.py ..." bash tools/gpu_quick.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${DQ_TAG:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${DQ_TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --skip-cpu-baseline ${DQ_BENCH_ARGS:-} > $OUT/bench.log 2>&1
