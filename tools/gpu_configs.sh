#!/bin/bash
# GPU box: bench lines for the secondary BASELINE configs (base f16 B=1, small bf16 B=32,
# large-v3-turbo bf16 B=256), one GPU each step with its own time limit; a failure ends the run.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
run() {
    local tag=$1; shift
    timeout -k 10 600 python bench.py "$@" > "gpurun_out/cfg_$tag.json" 2> "gpurun_out/cfg_$tag.err"
    local rc=$?; echo "$tag rc=$rc"; cat "gpurun_out/cfg_$tag.json"
    return $rc
}
run base_f16_b1 --model base --dtype f16 --batch 1 --steps 3 --warmup 1 &&
run small_bf16_b32 --model small --batch 32 --steps 2 --warmup 1 &&
run turbo_bf16_b256 --model large-v3-turbo --batch 256 --steps 2 --warmup 1
