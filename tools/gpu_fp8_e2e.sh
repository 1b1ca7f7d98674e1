#!/bin/bash
# GPU box: fp8 tests (kernels + whole encoder), the full GPU suite, then large-v3-turbo fp8 B=256.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1
rc=$?; echo "fp8 pytest rc=$rc"; grep -E 'FAIL|Error|assert|fp8 encoder' gpurun_out/pytest_fp8.log | head -20; tail -2 gpurun_out/pytest_fp8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --model large-v3-turbo --dtype fp8 --batch 256 --cpu-baseline 0 > gpurun_out/cfg_turbo_fp8_b256.json 2> gpurun_out/cfg_turbo_fp8_b256.err
rc=$?; echo "turbo fp8 rc=$rc"; cat gpurun_out/cfg_turbo_fp8_b256.json; tail -3 gpurun_out/cfg_turbo_fp8_b256.err; exit $rc
