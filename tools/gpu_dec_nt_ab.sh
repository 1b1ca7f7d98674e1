#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for v in 1 0 1 0; do
  timeout -k 10 400 env WHISPER_MI355X_DEC_NT=$v python bench.py --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 > gpurun_out/kt_$v.log 2> gpurun_out/kt_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/kt_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('DEC_NT=$v', d['value'], r['avg_launch_ms'], r['frac'], d['extra']['phase_ms_last_step'])"
done
