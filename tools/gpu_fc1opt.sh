# fc1's Adam in its weight-gradient epilogue (DQ_FC1_EPI_OPT=1, in-tree) vs the Adam riders
# (ab/fc1old): the CNN / agent / north-star tests, then the bench A/B, then a step timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/fc1opt
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_agent.py tests/test_gpu_northstar.py -m gpu -v --timeout 600 --timeout-method thread -k "not iqn" > $OUT/tests.log 2>&1
echo "tests rc=$?"; tail -2 $OUT/tests.log; grep -E "FAILED" $OUT/tests.log | head
bash tools/ab_lib.sh ab/fc1old/libdopamine_amd.so 2>&1 | cut -c1-60
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/pf -o run -- python3 bench.py --skip-cpu-baseline --skip-configs > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/pf/run_results.db k_c51 30 > $OUT/step_timeline.txt && cat $OUT/step_timeline.txt
