#!/bin/bash
# round 6: persistent encoder GEMM tiles (WHISPER_MI355X_GEMM_PS / variant 15): bitwise A/B on the encoder shapes,
# kernel / encoder parity with PS, headline bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
DV_VARIANTS="-1,15" timeout -k 10 300 python -u tools/gemm_dv_ab.py > gpurun_out/r06_gemm_ps_ab.txt 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/r06_gemm_ps_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_gemm_ps_ab.txt
WHISPER_MI355X_GEMM_PS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_parity.py \
    > gpurun_out/r06_ps_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r06_ps_tests.txt; exit 1; }
tail -2 gpurun_out/r06_ps_tests.txt
BENCH_ARGS="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="base GEMM_PS=1 base GEMM_PS=1" OUTP=r06_psab bash tools/gpu_envab.sh
