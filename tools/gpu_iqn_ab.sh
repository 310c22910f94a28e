# IQN (config 5): the IQN parity tests on the in-tree library, then config 5's step rate
# alternating in-tree / the given A/B builds, then a rocprofv3 kernel summary of the
# in-tree step.
#   gpurun -- bash tools/gpu_iqn_ab.sh <out-name> ab/X/libdopamine_amd.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-iqn_ab}
shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_iqn.py tests/test_gpu_northstar.py -k iqn -v \
  --timeout 300 --timeout-method thread > $OUT/iqn_tests.log 2>&1
rc=$?
tail -3 $OUT/iqn_tests.log
grep northstar_errors $OUT/iqn_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for lib in "" "$@"; do
    line=$(DOPAMINE_AMD_LIB=$lib timeout -k 10 200 python tools/bench_configs.py 300 iqn_breakout 2>>$OUT/ab_err.log | tail -1) || exit 1
    echo "[${lib:-in-tree}] $line" | tee -a $OUT/ab.log
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 tools/bench_configs.py 150 iqn_breakout pipeline=0 > $OUT/prof.log 2>&1 && \
python3 tools/prof_summary.py /tmp/prof/run_results.db 25 > $OUT/kernel_summary.txt
