#!/bin/bash
# Round-2 measurement pass (GPU box), each step under its own time limit, chained so that a failure
# ends the run: default bench line (CPU baseline, variants, front-end), rocprofv3 kernel stats of a
# short bench, PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and MFMA busy, then the secondary
# BASELINE config lines. Outputs under gpurun_out/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export NW_MODEL_DIR=/tmp/nw_models
step() { echo "== $1"; }
step bench && timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/m_bench.json 2> gpurun_out/m_bench.err &&
  tail -c 400 gpurun_out/m_bench.json &&
step prof && BENCH_ARGS="--tokens 32 --steps 1 --warmup 1 --cpu-baseline 0 --variants 0 --frontend 0" bash tools/gpu_prof.sh &&
step pmc && PMC_REGEX="xattn_step_kernel|gemm8p_kernel|gemm8p_mx_kernel|attn_enc2_kernel|gemm_dec_kernel|logits_kernel" bash tools/pmc.sh &&
python3 tools/pmc_traffic.py r02 > gpurun_out/m_pmc_traffic.txt 2>&1; tail -5 gpurun_out/m_pmc_traffic.txt
[ -n "$NO_MFMA" ] || { step mfma && bash tools/pmc_mfma.sh > gpurun_out/m_mfma.txt 2>&1; tail -12 gpurun_out/m_mfma.txt; }
[ -n "$NO_CFG" ] || {
  cd "$R"
  run() {
    local tag=$1; shift
    timeout -k 10 600 python3 bench.py --variants 0 --frontend 0 "$@" > "gpurun_out/cfg_$tag.json" 2> "gpurun_out/cfg_$tag.err"
    local rc=$?; echo "$tag rc=$rc"; tail -c 300 "gpurun_out/cfg_$tag.json"; return $rc
  }
  step cfg && run base_f16_b1 --model base --dtype f16 --batch 1 --steps 3 --warmup 1 &&
  run small_bf16_b32 --model small --batch 32 --steps 2 --warmup 1 &&
  run turbo_bf16_b256 --model large-v3-turbo --batch 256 --steps 2 --warmup 1 --cpu-baseline 0 &&
  run turbo_fp8_b256 --model large-v3-turbo --dtype fp8 --batch 256 --steps 2 --warmup 1 --cpu-baseline 0
}
