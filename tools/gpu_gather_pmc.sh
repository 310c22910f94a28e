# PMC traffic passes for the gather kernel (bash tools/gpu_gather_pmc.sh <out-name>) (one counter per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-gather_pmc}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/gather_traffic.py > $OUT/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/gather_traffic.py > $OUT/write.log 2>&1 && \
python3 tools/gather_traffic.py --summarize $OUT > $OUT/traffic.json
