#!/bin/bash
# round 6: encoder attention output rows staged through LDS (WHISPER_MI355X_ENC_ATTN_STG): bitwise variant test with
# the switch on, headline A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
WHISPER_MI355X_ENC_ATTN_STG=1 timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attn_encoder" > gpurun_out/r06_eastg_tests.txt 2>&1 || { tail -20 gpurun_out/r06_eastg_tests.txt; exit 1; }
grep -E "attn_encoder 32|passed|failed" gpurun_out/r06_eastg_tests.txt
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
BENCH_ARGS="$X" AB="base ENC_ATTN_STG=1 base ENC_ATTN_STG=1" OUTP=r06_eastg bash tools/gpu_envab.sh
