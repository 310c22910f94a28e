# A/B on one box: optional k_c51 stamps of a -DDQ_C51_PROF variant, chosen GPU tests, then
# alternating bench runs of the in-tree library and the named variants.
#   DQ_TAG=name DQ_TESTS="tests/a.py" DQ_STAMPS=ab/c51prof/libdopamine_amd.so \
#   gpurun -- bash tools/gpu_ab.sh ab/base/libdopamine_amd.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${DQ_TAG:-ab}
mkdir -p $OUT
if [ -n "$DQ_STAMPS" ]; then
  DOPAMINE_AMD_LIB=$DQ_STAMPS timeout -k 10 200 python -u tools/c51_stamps.py > $OUT/stamps.log 2>&1 || exit $?
  tail -12 $OUT/stamps.log
fi
if [ -n "$DQ_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $DQ_TESTS -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; grep FAILED $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
fi
bash tools/ab_lib.sh "$@" 2>&1 | tee $OUT/ab.log
