set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_c12
mkdir -p $O
PEER_IDLE_RANK=1 GP_POLLS=20000 timeout -k 10 100 python3 -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 tools/peer_smoke.py 4 > $O/smoke_idle.log 2>&1; echo "rc=$?"
grep -v "^\[W\|Gloo\|amdgpu.ids" $O/smoke_idle.log | tail -40
