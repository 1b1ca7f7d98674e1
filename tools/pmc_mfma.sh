#!/bin/bash
# MFMA-busy evidence for the MFMA-bound kernels (GPU box): one rocprofv3 --pmc pass per workload with
# SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE and (round 6, VERDICT r5 "next" 4) the stall counters
# SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_LDS, SQ_LDS_BANK_CONFLICT
# (8 SQ + 1 GRBM counters: one pass), counters only, each under its own time limit: large-v3 bf16 (gemm8p,
# attn_enc2) and large-v3-turbo fp8 (gemm8p_mx).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
REGEX="gemm8p_kernel|gemm8p_mx_kernel|attn_enc2_kernel"
run() {
  local tag=$1; shift
  local d="$R/gpurun_out/pmc_mfma_$tag"
  timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex "$REGEX" \
      --output-format csv -d "$d" -o run -- python3 "$R/bench.py" "$@" > "$d.log" 2>&1
  local rc=$?; echo "pmc $tag rc=$rc"; tail -2 "$d.log"; return $rc
}
X="--variants 0 --inflight-line 0 --f16-line 0 --frontend 0 --app-pattern 0 --cpu-baseline 0"
run bf16 --batch 32 --tokens 4 --steps 1 --warmup 1 $X &&
run fp8 --model large-v3-turbo --dtype fp8 --batch 32 --tokens 4 --steps 1 --warmup 1 $X &&
python3 "$R/tools/pmc_mfma.py" "${1:-r02}"
