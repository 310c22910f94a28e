set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_c14
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_peer.py -v --timeout 600 --timeout-method thread > $O/peer_tests.log 2>&1 || { echo "peer tests rc=$?"; tail -40 $O/peer_tests.log; exit 1; }
tail -3 $O/peer_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rd -o run -- python3 bench.py --force-dist --schedules peer --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 > $O/prof_peer.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof_peer.log; exit 1; }
python3 tools/step_timeline_db.py /tmp/rd/run_results.db k_c51 30 > $O/peer_step_timeline.txt; head -3 $O/peer_step_timeline.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "gpu tests rc=$?"; tail -5 $O/gpu_tests.log
