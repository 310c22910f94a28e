# IQN epilogue loads issued together (EpiDxQ's emb / state groups, EpiEmb's bias / state
# rows via HasVPre) vs the previous library (libdopamine_amd_prev.so): tests, same-box
# alternating config-5 lines, the one-stream timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2s5e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_iqn.py tests/test_gpu_cnn.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/new.log || exit 1
  DOPAMINE_AMD_LIB=$PWD/dopamine_amd/libdopamine_amd_prev.so timeout -k 10 200 python -u tools/bench_configs.py 150 iqn_breakout 2>&1 | tail -1 >> $OUT/prev.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof5 -o run -- python3 tools/bench_configs.py 150 iqn_breakout pipeline=0 > $OUT/prof.log 2>&1 && \
python3 tools/step_timeline_db.py /tmp/prof5/run_results.db k_iqn 30 > $OUT/step_timeline_one_stream.txt
