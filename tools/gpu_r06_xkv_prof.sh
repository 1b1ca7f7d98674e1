#!/bin/bash
# round 6: kernel summaries of the prompted variant lines, single cross K/V launch vs per layer
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for spec in 0 1; do
  rm -rf gpurun_out/prof
  WHISPER_MI355X_XKV_SPLIT=$spec BENCH_ARGS="--variants 1 --variant-steps 1 --fallback-line 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 1 --warmup 1" \
    bash tools/gpu_prof.sh > gpurun_out/prof_xkv$spec.log 2>&1 || { tail -5 gpurun_out/prof_xkv$spec.log; exit 1; }
  mv gpurun_out/prof_summary.md gpurun_out/r06_xkv_split${spec}_kernels.md; rm -rf gpurun_out/prof
  echo "== XKV_SPLIT=$spec"; grep -E "gemm8p_kernelIDF16bLi5|attn_prefill|gemm_glds|gemm8p_kernelIDF16bLi[0-4]" gpurun_out/r06_xkv_split${spec}_kernels.md | cut -c1-150
done
