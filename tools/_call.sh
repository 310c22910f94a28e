set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_c12
mkdir -p $O
GP_POLLS=100000 timeout -k 10 100 python3 -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 tools/peer_smoke.py 4 > $O/smoke2.log 2>&1; echo "rc=$?"; grep -v "^\[W\|Gloo\|amdgpu.ids" $O/smoke2.log | tail -12
PEER_IDLE_RANK=1 GP_POLLS=20000 timeout -k 10 100 python3 -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 tools/peer_smoke.py 4 > $O/smoke_idle.log 2>&1; echo "rc=$?"
grep -v "^\[W\|Gloo\|amdgpu.ids" $O/smoke_idle.log | tail -40
timeout -k 10 600 python -u -m pytest tests/test_gpu_iqn.py -v --timeout 300 --timeout-method thread -k "fused_optimizer" > $O/iqn_fused.log 2>&1; echo "iqn rc=$?"
grep -E "PASSED|FAILED|passed|failed|Error" $O/iqn_fused.log | tail -12
for rep in 1 2; do
  for extra in "" "--force-dist --schedules peer"; do
    line=$(timeout -k 10 240 python bench.py --steps 2000 --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 $extra 2>>$O/err.log | tail -1) || exit 1
    echo "[${extra:-no group}] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["parallelism"])')" | tee -a $O/one_rank_ab.log
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rd -o run -- python3 bench.py --force-dist --schedules peer --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 > $O/prof_peer.log 2>&1 || exit 1
python3 tools/step_timeline_db.py /tmp/rd/run_results.db k_c51 30 > $O/peer_step_timeline.txt; cat $O/peer_step_timeline.txt
