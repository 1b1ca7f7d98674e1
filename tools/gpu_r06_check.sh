#!/bin/bash
# round 6: the reverted encoder GEMM: isolated shapes and the headline bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
DV_VARIANTS="-1" timeout -k 10 300 python -u tools/gemm_dv_ab.py > gpurun_out/r06_gemm_check.txt 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/r06_gemm_check.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_gemm_check.txt
BENCH_ARGS="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="base ENC_BATCH=32 base" OUTP=r06_check bash tools/gpu_envab.sh
