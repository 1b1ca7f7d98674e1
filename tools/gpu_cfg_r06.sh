#!/bin/bash
# Round-6 lines of the BASELINE configs and the strong-scaling shards on the final build (1 GPU; each run has
# its own time limit, a failure ends the script): gpurun_out/r06_cfg_<tag>.json
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0"
run() {
    local tag=$1; shift
    timeout -k 10 400 python bench.py $X "$@" > "gpurun_out/r06_cfg_$tag.json" 2> "gpurun_out/r06_cfg_$tag.err" || { echo "$tag FAIL"; tail -3 "gpurun_out/r06_cfg_$tag.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r06_cfg_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['extra']['phase_ms_last_step'], 'give_ups', d['extra'].get('pdec_give_ups'))"
}
run base_f16_b1 --model base --dtype f16 --global-batch 1 --steps 3 &&
run lv3_f16_b1 --model large-v3 --dtype f16 --global-batch 1 --steps 2 &&
run small_bf16_b32 --model small --global-batch 32 --steps 2 &&
run turbo_fp8_b256 --model large-v3-turbo --dtype fp8 --global-batch 256 --steps 2 &&
run lv3_b64 --global-batch 64 --steps 2 &&
run lv3_b32 --global-batch 32 --steps 2 &&
run lv3_b16 --global-batch 16 --steps 2
