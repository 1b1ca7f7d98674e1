cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=3,-1 timeout -k 10 300 python tools/gemm_tune.py --bf16 > gpurun_out/gt.log 2>&1; rc=$?; cat gpurun_out/gt.log; exit $rc
