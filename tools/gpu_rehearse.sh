# N > 1 on ONE GPU: the peer exchange's tests, then bench.py's whole N-rank path with every
# rank on cuda:0 over gloo (DQ_BENCH_REHEARSE=1), printing the N > 1 line's self-checks
# (replicas compared bit for bit, self-test verdict, per-rank waits at each exchange point).
#   gpurun -- bash tools/gpu_rehearse.sh <out-name> <what>
# what: tests | w2 | w4 | w8 | faults | replica (a comma list).  replica: the variant whose
# rank 1 computes its replicated conv-bucket mean 2^-20 off (its replica must be caught).  faults: world-2 rehearsals on the
# fault-injection variants (variants/, built here by tools/build_variant.py with
# DQ_VARIANT_ROOT=variants): one XCD's blocks hidden from the publication's count, one XCD's
# write-back dropped (self-test on, then off so that only the replica check can catch it).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-rehearse}
WHAT=${2:-tests,w2}
mkdir -p $OUT
port=29611
bench_n() {   # world, log name, extra env...
  local n=$1 log=$2
  shift 2
  port=$((port + 1))
  env DQ_BENCH_REHEARSE=1 "$@" timeout -k 10 560 python -u -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n \
      --steps 20 --warmup 5 > $OUT/$log.log 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  grep -E '^\{' $OUT/$log.log | tail -1 | python3 -c '
import sys, json
d = json.loads(sys.stdin.read())
print("headline", d["value"], d["config"]["parallelism"])
for k, v in (d.get("schedules") or {}).items():
  print(" ", k, json.dumps(v)[:1500])' || grep -E "bench:|Error|error" $OUT/$log.log | tail -5
  return $rc
}
if [[ $WHAT == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_peer.py -m gpu -v -s --timeout 600 \
      --timeout-method thread > $OUT/peer_tests.log 2>&1
  rc=$?; echo "peer tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^selftest" $OUT/peer_tests.log | tail -20
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
for w in 2 4 8; do
  if [[ $WHAT == *w$w* ]]; then bench_n $w rehearse_w$w || exit $?; fi
done
if [[ $WHAT == *replica* ]]; then
  bench_n 2 fault_replica DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=variants/peer_fault_replica/libdopamine_amd.so || exit $?
fi
if [[ $WHAT == *faults* ]]; then
  bench_n 2 fault_hide_xcd DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=variants/peer_hide_xcd/libdopamine_amd.so || exit $?
  bench_n 2 fault_drop_fence DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=variants/peer_drop_fence/libdopamine_amd.so || exit $?
  bench_n 2 fault_drop_fence_no_selftest DQ_DIAGNOSTIC_BUILD=1 DQ_PEER_SKIP_SELFTEST=1 DOPAMINE_AMD_LIB=variants/peer_drop_fence/libdopamine_amd.so || exit $?
fi
exit 0
