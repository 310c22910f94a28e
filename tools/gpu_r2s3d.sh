# the default bench line (headline + configs 2/5 + CPU baseline), then the two-rank gloo rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3d
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2> $OUT/bench.err && \
DQ_BENCH_REHEARSE=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 100 > $OUT/rehearse.log 2>&1
