# Split-bf16 ("x6") GEMM form vs exact f32: per library, the IQN executor's float64 errors
# (printed), then config 5 alternating over the libraries, then (if given) the Rainbow
# CNN tests + bench for the CNN variant.
#   gpurun -- bash tools/gpu_x6_ab.sh <out-name> "<iqn libs>" "<cnn lib or empty>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-x6_ab}
mkdir -p $OUT
for lib in $2; do
  DOPAMINE_AMD_LIB=$lib timeout -k 10 200 python -u -m pytest "tests/test_gpu_iqn.py::test_iqn_executor_matches_float64" \
    -s -q --timeout 150 --timeout-method thread > $OUT/errs_$(basename $(dirname $lib)).log 2>&1
  rc=$?
  echo "[$lib] rc=$rc"; grep "grad errors" $OUT/errs_$(basename $(dirname $lib)).log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for rep in 1 2; do
  for lib in $2; do
    line=$(DOPAMINE_AMD_LIB=$lib timeout -k 10 200 python tools/bench_configs.py 300 iqn_breakout 2>>$OUT/ab_err.log | tail -1) || exit 1
    echo "[$lib] $line" | tee -a $OUT/ab.log
  done
done
if [ -n "$3" ]; then
  DOPAMINE_AMD_LIB=$3 timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_northstar.py -k "not iqn" -q \
    --timeout 300 --timeout-method thread > $OUT/cnn_tests.log 2>&1
  rc=$?
  tail -3 $OUT/cnn_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  bash tools/ab_lib.sh $3 | tee $OUT/rainbow_ab.log
fi
