#!/bin/bash
# round 6: the cache-form cross step at 16 / 32 clips with the 1024-thread kernel (XWIDE_MAX) vs the 256-thread one
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
for b in ${XW_BATCHES:-16 32}; do
  BENCH_ARGS="$X --global-batch $b" AB="${XW_AB:-base XWIDE_MAX=32 base XWIDE_MAX=32}" OUTP=r06_xw_b$b bash tools/gpu_envab.sh || exit 1
done
