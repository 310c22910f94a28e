set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_c2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u tools/window_probe.py 20 300 > $O/window_probe.log 2>&1 || exit $?
cat $O/window_probe.log | tail -4
DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=ab/gprof/libdopamine_amd.so timeout -k 10 300 python3 -u tools/gather_stamps.py > $O/gather_stamps.log 2>&1 || exit $?
tail -16 $O/gather_stamps.log
timeout -k 10 300 python3 -u tools/dist_graph_dot.py $O/dist_dot > $O/dist_dot.log 2>&1; echo "dot rc=$?"
tail -3 $O/dist_dot.log
