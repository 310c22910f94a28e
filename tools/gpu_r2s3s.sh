# IQN split Adam: IQN tests + same-box A/B; then the N > 1 fc-update stream placement A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3s
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_iqn.py tests/test_gpu_agent.py tests/test_gpu_northstar.py tests/test_gpu_agent_api.py -m gpu -v --timeout 240 --timeout-method thread -k "iqn" > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/iqn_adam_ab.py > $OUT/iqn_ab.log 2>&1 && \
bash tools/gpu_r2s3r.sh
