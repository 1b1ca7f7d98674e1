#!/bin/bash
# Round 3, pass D: where the decode step's time goes. Same-box env A/Bs of the headline bench (128 clips)
# and of one 16-clip shard: DBG_SAMEW=1 (every decoder layer reads layer 0's weights: the upper bound of
# any weight prefetch), XKEEP=k (the first k clips' encoder rows with the default cache policy: MALL
# residency across decoder layers), DEC_NT=0 (decode weights with the default policy).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
AB="${AB128:-base DBG_SAMEW=1 PREFETCH=64 PREFETCH=160 XKEEP=32 XKEEP=64 DEC_NT=0 base}" OUTP=ab128 bash tools/gpu_envab.sh || exit $?
AB="${AB16:-base DBG_SAMEW=1 PREFETCH=64 base}" OUTP=ab16 \
  BENCH_ARGS="--global-batch 16 --steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0" \
  bash tools/gpu_envab.sh || exit $?
