#!/bin/bash
# round 6: cross K/V epilogue with whole-row stores: isolated timing, bitwise against the previous build's logits
# (16-clip cache form), then the prompted variants and the 16-clip line
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug/xkv_shape.py 2>&1 | grep -v amdgpu.ids || exit 1
cp tools/debug/ref/envlg_x16_r06pre.npy gpurun_out/envlg_pre.npy
timeout -k 10 200 python -u tools/debug/env_logits.py x16new 16 cache || exit 1
python tools/debug/env_logits.py --compare pre x16new || exit 1
rm -f gpurun_out/envlg_pre.npy gpurun_out/envlg_x16new.npy
V="--variants 1 --variant-steps 2 --fallback-line 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 1"
timeout -k 10 400 python -u bench.py $V > gpurun_out/r06_xkv3_var.json 2> gpurun_out/r06_xkv3_var.err || { tail -3 gpurun_out/r06_xkv3_var.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r06_xkv3_var.json').read().strip().splitlines()[-1])
print('headline', d['value'], d['extra']['phase_ms_last_step'])
for v in d['variants'][:3]: print(v['workload'][:40], v['value'], v.get('phase_ms_last_step'))"
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
BENCH_ARGS="$X --global-batch 16" AB="base base" OUTP=r06_xkv3_b16 bash tools/gpu_envab.sh || exit 1
