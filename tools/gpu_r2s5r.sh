# The N > 1 bench path at HEAD: a two-rank gloo rehearsal on one GPU (init, per-rank fill,
# split graphs, barriers, max-over-ranks timing, the JSON line) and the one-rank RCCL line
# (--force-dist: every collective executed, captured in the chunk graphs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5r
mkdir -p $OUT
DQ_BENCH_REHEARSE=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 100 > $OUT/rehearse.log 2>&1 && \
timeout -k 10 300 python -u bench.py --force-dist --skip-cpu-baseline --steps 1000 > $OUT/force_dist.log 2>&1
