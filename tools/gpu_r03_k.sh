#!/bin/bash
# Round 3, pass K: whole -m gpu suite; A/B of the split logits kernels at 1 and 16 clips.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03k_all.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r03k_all.log | tail -8; [ $rc -le 1 ] || exit $rc
X="--variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0"
AB="LOGITS_SPLIT_MAX=0 base LOGITS_SPLIT_MAX=0 base" OUTP=abls BENCH_ARGS="--model base --dtype f16 --global-batch 1 --steps 10 --warmup 2 $X" bash tools/gpu_envab.sh || exit $?
AB="LOGITS_SPLIT_MAX=0 base" OUTP=abls16 BENCH_ARGS="--global-batch 16 --steps 2 --warmup 1 $X" bash tools/gpu_envab.sh || exit $?
