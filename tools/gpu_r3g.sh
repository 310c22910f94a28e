# Chunk gather (uniform replay learner loop): agent tests, the DQN north-star lockstep, the
# bench line (config 2 with its chunk-gather roofline), IQN stream-priority A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_northstar.py -m gpu -v --timeout 600 --timeout-method thread -k "not iqn" > $OUT/tests.log 2>&1
echo "tests rc=$?"; grep -E "PASSED|FAILED|Error" $OUT/tests.log | cut -c1-160 | tail -40
timeout -k 10 400 python -u bench.py --skip-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], json.dumps(d["other_configs"]))'
for rep in 1 2; do
  for pr in none main:-1; do
    timeout -k 10 300 python -u tools/iqn_priority.py $pr 150 2>&1 | tail -1 || exit 1
  done
done
