#!/bin/bash
# round 6: the coalesced encoder GEMM epilogue (default): kernel / encoder parity, clock stamps, headline bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_parity.py \
    > gpurun_out/r06_gemm4_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r06_gemm4_tests.txt; exit 1; }
tail -2 gpurun_out/r06_gemm4_tests.txt
timeout -k 10 200 python -u tools/gemm_stamps.py > gpurun_out/r06_gemm_stamps_coal.txt 2>&1 || { echo "stamps rc=$?"; tail -5 gpurun_out/r06_gemm_stamps_coal.txt; exit 1; }
cat gpurun_out/r06_gemm_stamps_coal.txt
BENCH_ARGS="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="base base" OUTP=r06_coal bash tools/gpu_envab.sh
