#!/bin/bash
# Round 3: bench lines of the other BASELINE configs and of the strong-scaling shards (large-v3 bf16 at
# 64 / 32 / 16 clips = one rank's share of the 128-clip batch at 2 / 4 / 8 GPUs), one step each under
# its own time limit; a failure ends the run.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
X="--variants 0 --frontend 0 --app-pattern 0"
run() {
    local tag=$1; shift
    timeout -k 10 600 python bench.py "$@" > "gpurun_out/cfgc_$tag.json" 2> "gpurun_out/cfgc_$tag.err"
    local rc=$?; echo "$tag rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "gpurun_out/cfgc_$tag.err"; return $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/cfgc_$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('  ', d['value'], d['extra']['phase_ms_last_step'], r['kernel'], r['frac'], (d.get('cpu_baseline') or {}).get('value'))"
}
run base_f16_b1 --model base --dtype f16 --global-batch 1 --steps 10 --warmup 2 $X &&
run small_bf16_b32 --model small --global-batch 32 --steps 2 --warmup 1 $X &&
run turbo_bf16_b256 --model large-v3-turbo --global-batch 256 --steps 2 --warmup 1 $X &&
run turbo_fp8_b256 --model large-v3-turbo --dtype fp8 --global-batch 256 --steps 2 --warmup 1 $X --cpu-baseline 0 &&
run largev3_b64 --global-batch 64 --steps 2 --warmup 1 $X --cpu-baseline 0 &&
run largev3_b32 --global-batch 32 --steps 2 --warmup 1 $X --cpu-baseline 0 &&
run largev3_b16 --global-batch 16 --steps 3 --warmup 1 $X --cpu-baseline 0
