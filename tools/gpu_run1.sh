cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xattn.py tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.log
exit $rc
