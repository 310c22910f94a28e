# IQN FC1 split in whole rounds: IQN tests, then same-box A/B against the previous library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_iqn.py tests/test_gpu_northstar.py -m gpu -v --timeout 240 --timeout-method thread -k "iqn" > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/new.log || exit 1
  DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdq_ref.so timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/ref.log || exit 1
done
