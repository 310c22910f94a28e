# one-rank RCCL schedule: the fc update on the comm stream vs on the second stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3r
mkdir -p $OUT
for i in 1 2; do
timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --force-dist --steps 600 --gather-iters 20 2>&1 | tail -1 | cut -c1-120 >> $OUT/one_stream.log || exit 1
DQ_EXP_FC_OPT_STREAM=1 timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --force-dist --steps 600 --gather-iters 20 2>&1 | tail -1 | cut -c1-120 >> $OUT/two_streams.log || exit 1
done
