#!/bin/bash
# round 6: self-attention decode step, heads per workgroup (4 / 2 / 1) at 128 and 16 clips
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
for b in ${HPB_BATCHES:-128 16}; do
  BENCH_ARGS="$X --global-batch $b" AB="base SELF_HPB=2 SELF_HPB=1 base SELF_HPB=2 SELF_HPB=1" OUTP=r06_hpb_b$b bash tools/gpu_envab.sh || exit 1
done
