#!/bin/bash
# HBM traffic of the roofline kernels from PMC counters (GPU box). Two separate passes, FETCH_SIZE
# and WRITE_SIZE (they do not fit one TCC pass), counters only (no sys/runtime trace), each on a
# short bench run (same per-launch work as the full bench: cross-attention always reads 1500 keys).
# Output: gpurun_out/pmc_{fetch,write}/ CSVs; tools/pmc_traffic.py turns them into bytes/launch.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
# BATCHES: one pass pair per global batch (the strong-scaling shards: 128 / 64 / 32 / 16 clips per GPU
# at 1 / 2 / 4 / 8 GPUs; up to 32 clips the cached cross form runs attn_cross_step_kernel)
ARGS="--tokens 4 --steps 1 --warmup 1 --cpu-baseline 0 --variants 0 --frontend 0 --app-pattern 0 ${PMC_ARGS}"
REGEX="${PMC_REGEX:-xattn_step_kernel|attn_cross_step|gemm8p_kernel|attn_enc2_kernel|gemm_dec_kernel|splitk_reduce|pdec_kernel|gemm_small_kernel}"
for B in ${BATCHES:-128}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d="$R/gpurun_out/pmc_$(echo $c | tr A-Z a-z | cut -d_ -f1)_b$B"
    timeout -k 10 ${T_PMC:-500} rocprofv3 --pmc $c --kernel-include-regex "$REGEX" --output-format csv -d "$d" -o run \
        -- python3 "$R/bench.py" $ARGS --global-batch $B > "$d.log" 2>&1
    rc=$?; echo "pmc $c B=$B rc=$rc"; tail -2 "$d.log"
    [ $rc -eq 0 ] || exit $rc
  done
done
