#!/bin/bash
# rocprofv3 kernel summaries of the decode path at a small shard (16 clips: one rank of configs[3] at
# 8 GPUs), split-K path (SMALLM=0) vs the small-M path (SMALLM=1), same box.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
for v in ${VARIANTS:-0 1}; do
  rm -rf gpurun_out/prof
  WHISPER_MI355X_SMALLM=$v BENCH_ARGS="--global-batch ${NB:-16} --tokens 32 --steps 1 --warmup 1 --cpu-baseline 0 --variants 0 --frontend 0 --app-pattern 0" \
    bash tools/gpu_prof.sh > gpurun_out/prof16_$v.log 2>&1 || { cat gpurun_out/prof16_$v.log; exit 1; }
  mv gpurun_out/prof_summary.md gpurun_out/prof${NB:-16}_smallm$v.md
  echo "== SMALLM=$v"; head -30 gpurun_out/prof${NB:-16}_smallm$v.md
done
