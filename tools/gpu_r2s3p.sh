# ZeRO-1 in the captured chunk graphs (experiment): the one-rank RCCL bench with capture on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s3p
mkdir -p $OUT
DQ_EXP_ZERO_CAPTURE=1 timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --force-dist --zero 1 --steps 400 --gather-iters 20 > $OUT/fd_zero_capture.log 2>&1
echo "rc=$?"
timeout -k 10 300 python -u bench.py --skip-cpu-baseline --skip-configs --force-dist --zero 1 --steps 400 --gather-iters 20 > $OUT/fd_zero.log 2>&1
