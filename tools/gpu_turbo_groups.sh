#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for g in 1 2; do
  WHISPER_MI355X_DEC_STREAMS=$g timeout -k 10 600 python bench.py --model large-v3-turbo --dtype fp8 --batch 256 --cpu-baseline 0 > gpurun_out/turbo_g$g.json 2> gpurun_out/turbo_g$g.err
  rc=$?; echo "groups=$g rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/turbo_g$g.json')); print(d['value'], d['extra']['phase_ms_last_step'])"
done
