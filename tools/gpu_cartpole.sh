cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
timeout -k 10 300 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_cartpole.py -v --timeout 240 --timeout-method thread > gpurun_out/r2a/cp.log 2>&1
