#!/bin/bash
# encoder windows per launch group (WHISPER_MI355X_ENC_BATCH) A/B at 128 clips
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for v in 32 64 128 32 128; do
  timeout -k 10 400 env WHISPER_MI355X_ENC_BATCH=$v python bench.py --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 > gpurun_out/encb_$v.log 2> gpurun_out/encb_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench encb=$v rc=$rc"; tail -5 gpurun_out/encb_$v.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/encb_$v.log').read().strip().splitlines()[-1]); print('encb=$v', d['value'], d['extra']['phase_ms_last_step'])"
done
