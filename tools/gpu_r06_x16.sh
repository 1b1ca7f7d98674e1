#!/bin/bash
# round 6: the 16/32-clip lines with the cross form forced each way, then a kernel summary of the 16-clip step
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
for b in 16 32; do
  BENCH_ARGS="$X --global-batch $b" AB="CROSS=cache CROSS=direct" OUTP=r06_x_b$b bash tools/gpu_envab.sh || exit 1
done
rm -rf gpurun_out/prof
BENCH_ARGS="--global-batch 16 --steps 1 --warmup 1 $X" bash tools/gpu_prof.sh > gpurun_out/prof16.log 2>&1 || { tail -5 gpurun_out/prof16.log; exit 1; }
mv gpurun_out/prof_summary.md gpurun_out/r06_prof16_kernels.md; rm -rf gpurun_out/prof
head -40 gpurun_out/r06_prof16_kernels.md
