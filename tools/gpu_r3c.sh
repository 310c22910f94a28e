set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_roofline.sh r3_roofline || exit 1
OUT=gpurun_out/r3_capture; mkdir -p $OUT
timeout -k 10 60 ./tools/micro/capture_fork.bin 1 > $OUT/hip_1.log 2>&1; rc=$?; echo "hip 1 rc=$rc"; cat $OUT/hip_1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 60 ./tools/micro/capture_fork.bin 4 > $OUT/hip_4.log 2>&1; rc=$?; echo "hip 4 rc=$rc"; cat $OUT/hip_4.log; [ $rc -eq 0 ] || exit 1
AMD_LOG_LEVEL=4 timeout -k 10 120 python -u tools/capture_fork_repro.py 1 plain > $OUT/torch_1_log4.log 2>&1; echo "torch 1 rc=$?"
tail -40 $OUT/torch_1_log4.log | cut -c1-300
