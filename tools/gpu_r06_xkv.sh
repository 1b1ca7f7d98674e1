#!/bin/bash
# round 6: cross K/V GEMM split per decoder layer: bitwise check (16-clip cache form), then the 16-clip line and the
# prompted variants at 128 clips, single launch (XKV_SPLIT=0) vs per layer
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/debug/env_logits.py x16 16 cache || exit 1
WHISPER_MI355X_XKV_SPLIT=0 timeout -k 10 200 python -u tools/debug/env_logits.py x16_one 16 cache || exit 1
python tools/debug/env_logits.py --compare x16 x16_one || exit 1
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
BENCH_ARGS="$X --global-batch 16" AB="XKV_SPLIT=0 base XKV_SPLIT=0 base" OUTP=r06_xkv_b16 bash tools/gpu_envab.sh || exit 1
V="--variants 1 --variant-steps 2 --fallback-line 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 1"
for spec in XKV_SPLIT=0 base; do
  envs=(); [ "$spec" != base ] && envs=("WHISPER_MI355X_$spec")
  timeout -k 10 400 env "${envs[@]}" python -u bench.py $V > gpurun_out/r06_xkv_var_$spec.json 2> gpurun_out/r06_xkv_var_$spec.err || { echo "$spec rc=$?"; tail -3 gpurun_out/r06_xkv_var_$spec.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06_xkv_var_$spec.json').read().strip().splitlines()[-1])
for v in d['variants'][:3]: print('$spec', v['workload'][:40], v['value'], v.get('phase_ms_last_step'))"
done
