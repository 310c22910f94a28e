# Rainbow A/B: the CNN / north-star parity tests on each given build, then the bench
# alternating in-tree / builds (tools/ab_lib.sh) and a rocprof step timeline of each build.
#   gpurun -- bash tools/gpu_rainbow_ab.sh <out-name> ab/X/libdopamine_amd.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-rainbow_ab}
shift
mkdir -p $OUT
for lib in "$@"; do
  DOPAMINE_AMD_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_northstar.py tests/test_gpu_agent.py -k "not iqn" -q \
    --timeout 300 --timeout-method thread > $OUT/tests_$(basename $(dirname $lib)).log 2>&1
  rc=$?
  echo "[$lib] tests rc=$rc"; tail -1 $OUT/tests_$(basename $(dirname $lib)).log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
bash tools/ab_lib.sh "$@" | tee $OUT/ab.log
for lib in "$@"; do
  n=$(basename $(dirname $lib))
  DOPAMINE_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r_$n -o run -- python3 bench.py --skip-cpu-baseline --skip-configs > $OUT/prof_$n.log 2>&1 || exit 1
  python3 tools/step_timeline_db.py /tmp/r_$n/run_results.db k_c51 30 > $OUT/timeline_$n.txt
done
