# x6 numerics: the bf16-MFMA accumulation micro test, then the IQN executor's float64
# errors per library (printed).   gpurun -- bash tools/gpu_x6_num.sh <out> "<libs>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-x6_num}
mkdir -p $OUT
timeout -k 10 60 ./tools/micro/mfma_acc.bin | tee $OUT/mfma_acc.log || exit 1
for lib in $2; do
  DOPAMINE_AMD_LIB=$lib timeout -k 10 120 python -u tools/x6_dx_err.py 2>&1 | tail -1 | tee -a $OUT/dx_err.log || exit 1
done
for lib in $2; do
  DOPAMINE_AMD_LIB=$lib timeout -k 10 200 python -u -m pytest "tests/test_gpu_iqn.py::test_iqn_executor_matches_float64" \
    -s -q --timeout 150 --timeout-method thread > $OUT/errs_$(basename $(dirname $lib)).log 2>&1
  rc=$?
  echo "[$lib] rc=$rc"; grep "grad errors" $OUT/errs_$(basename $(dirname $lib)).log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for rep in 1 2; do
  for lib in $2; do
    line=$(DOPAMINE_AMD_LIB=$lib timeout -k 10 200 python tools/bench_configs.py 300 iqn_breakout 2>>$OUT/ab_err.log | tail -1) || exit 1
    echo "[$lib] $line" | tee -a $OUT/ab.log
  done
done
