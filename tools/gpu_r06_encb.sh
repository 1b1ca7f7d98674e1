#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
BENCH_ARGS="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="base ENC_BATCH=64 ENC_BATCH=128 base ENC_BATCH=128" OUTP=r06_encb bash tools/gpu_envab.sh
