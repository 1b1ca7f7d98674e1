#!/bin/bash
# round 6: encoder windows per launch group for the turbo fp8 line (256 clips)
set -o pipefail
cd "$(dirname "$0")/.."
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2 --model large-v3-turbo --dtype fp8 --global-batch 256"
BENCH_ARGS="$X" AB="base ENC_BATCH=32 ENC_BATCH=64 base ENC_BATCH=32 ENC_BATCH=64" OUTP=r06_encb_fp8 bash tools/gpu_envab.sh
