# one-rank RCCL schedule (bench --force-dist) under HIP graph queue knobs
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2e
mkdir -p $OUT
for cfg in "base" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
  env $e timeout -k 10 200 python -u bench.py --skip-cpu-baseline --steps 400 --force-dist --gather-iters 20 > $OUT/fd_$cfg.log 2>&1 || exit $?
  echo "$cfg $(tail -1 $OUT/fd_$cfg.log | cut -c1-160)"
done
