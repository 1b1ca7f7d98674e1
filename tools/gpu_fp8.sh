#!/bin/bash
# GPU box: fp8 kernel tests, then the fp8-vs-bf16 encoder GEMM timing.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'PASS|FAIL|Error|error|assert' gpurun_out/pytest_fp8.log | head -40; tail -3 gpurun_out/pytest_fp8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/fp8_gemm_bench.py > gpurun_out/fp8_bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/fp8_bench.txt; exit $rc
