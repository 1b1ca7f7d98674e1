#!/bin/bash
# round 6: (1) persistent encoder GEMM tiles v2 (next-tile DMA after the epilogue's first loads): bitwise A/B and
# headline bench A/B; (2) the fused logits combine (last-arriving workgroup): parity tests, base f16 1-clip A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
DV_VARIANTS="-1,15" timeout -k 10 300 python -u tools/gemm_dv_ab.py > gpurun_out/r06_gemm_ps_ab.txt 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/r06_gemm_ps_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_gemm_ps_ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pdec.py tests/test_gpu_pipe.py tests/test_gpu_parity.py \
    > gpurun_out/r06_logits_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r06_logits_tests.txt; exit 1; }
tail -2 gpurun_out/r06_logits_tests.txt
BENCH_ARGS="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="base GEMM_PS=1 base GEMM_PS=1" OUTP=r06_psab2 bash tools/gpu_envab.sh || exit 1
BENCH_ARGS="--model base --dtype f16 --global-batch 1 --steps 3 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="LOGITS_FUSED=0 base LOGITS_FUSED=0 base" OUTP=r06_lgab bash tools/gpu_envab.sh
