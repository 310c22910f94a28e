# Round-3 session checks: the new parity tests (C51 c51.gin, IQN double_dqn, IQN's bounded
# unpinned gradient), the fc-branch fork with a fake all-reduce, IQN stream priority A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_northstar.py -m gpu -v -s --timeout 600 --timeout-method thread > $OUT/northstar.log 2>&1
echo "northstar rc=$?"; grep -E "PASSED|FAILED|northstar_errors|Error" $OUT/northstar.log | cut -c1-400
for rep in 1 2; do
  timeout -k 10 300 python -u tools/dist_fake_ar.py --steps 2000 > $OUT/fake_ar_$rep.log 2>&1 || exit 1
  tail -1 $OUT/fake_ar_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("fake-ar", d["value"], d["ms_per_step"])'
done
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/pf -o run -- python3 tools/dist_fake_ar.py > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/pf/run_results.db k_c51 30 > $OUT/fake_ar_timeline.txt || exit 1
for rep in 1 2; do
  for pr in 0 -1; do
    timeout -k 10 300 python -u tools/iqn_priority.py $pr 150 2>&1 | tail -1 || exit 1
  done
done
