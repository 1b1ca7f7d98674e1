#!/bin/bash
# round 6: rocprofv3 kernel summary of the turbo fp8 256-clip line (configs[4])
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -rf gpurun_out/prof
BENCH_ARGS="--model large-v3-turbo --dtype fp8 --global-batch 256 --steps 1 --warmup 1 --variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0" \
  bash tools/gpu_prof.sh > gpurun_out/prof_fp8.log 2>&1 || { tail -5 gpurun_out/prof_fp8.log; exit 1; }
mv gpurun_out/prof_summary.md gpurun_out/r06_turbo_fp8_b256_kernels.md; rm -rf gpurun_out/prof
head -24 gpurun_out/r06_turbo_fp8_b256_kernels.md
