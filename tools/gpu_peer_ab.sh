# One-rank peer schedule A/B on one GPU: the peer tests on the product build, then alternating
# bench runs (no group / peer with a baseline library / peer with the product), then the
# product's peer step timeline.
#   gpurun -- bash tools/gpu_peer_ab.sh <out-name> <baseline-lib>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-peer_ab}
BASE=${2:-variants/head/libdopamine_amd.so}
mkdir -p $OUT
if [ -z "$DQ_AB_NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py -m gpu -v --timeout 500 --timeout-method thread > $OUT/peer_tests.log 2>&1
  rc=$?; echo "peer tests rc=$rc"; tail -3 $OUT/peer_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
B="--steps 2000 --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20"
row() {   # label, env, extra args
  line=$(env $2 timeout -k 10 240 python bench.py $B $3 2>>$OUT/err.log | tail -1) || return 1
  echo "[$1] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT/ab.log
}
for rep in 1 2 3; do
  row "no group" "" "" || exit 1
  row "peer base" "DOPAMINE_AMD_LIB=$BASE DQ_DIAGNOSTIC_BUILD=1" "--force-dist --schedules peer" || exit 1
  row "peer new" "" "--force-dist --schedules peer" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rd -o run -- python3 bench.py --force-dist --schedules peer --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 > $OUT/prof_peer.log 2>&1 || exit 1
python3 tools/step_timeline_db.py /tmp/rd/run_results.db k_c51 30 > $OUT/peer_step_timeline.txt
head -16 $OUT/peer_step_timeline.txt
