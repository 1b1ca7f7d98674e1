#!/bin/bash
# round 6: XCD-grouped encoder attention grid: bitwise + timing tests, then the headline bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attn_encoder" > gpurun_out/r06_eax_tests.txt 2>&1 || { tail -20 gpurun_out/r06_eax_tests.txt; exit 1; }
grep -E "attn_encoder 32|passed|failed" gpurun_out/r06_eax_tests.txt
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
BENCH_ARGS="$X" AB="${EAX_AB:-ENC_ATTN_XCD=0 base ENC_ATTN_XCD=0 base}" OUTP=r06_eax bash tools/gpu_envab.sh
