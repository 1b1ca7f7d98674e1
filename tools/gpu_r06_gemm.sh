#!/bin/bash
# round 6: encoder GEMM clock stamps (DV 0 and 2) and the headline bench with each LDS-DMA placement
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in 10 12; do
  timeout -k 10 200 python -u tools/gemm_stamps.py $v > gpurun_out/r06_gemm_stamps_$v.txt 2>&1 || { echo "stamps rc=$?"; tail -5 gpurun_out/r06_gemm_stamps_$v.txt; exit 1; }
  cat gpurun_out/r06_gemm_stamps_$v.txt
done
BENCH_ARGS="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="GEMM_DV=0 GEMM_DV=2 GEMM_DV=1 GEMM_DV=0 GEMM_DV=2" OUTP=r06_dvab bash tools/gpu_envab.sh
