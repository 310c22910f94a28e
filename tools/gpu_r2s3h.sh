# RNG-tape probe wait: refill counts, window spread, and the replay / agent GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3h
mkdir -p $OUT
timeout -k 10 300 python -u tools/tape_refills.py > $OUT/tape.log 2>&1 && \
timeout -k 10 300 python -u tools/window_spread.py 20 200 > $OUT/spread.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_api.py tests/test_gpu_agent.py tests/test_gpu_sumtree.py tests/test_gpu_northstar.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
