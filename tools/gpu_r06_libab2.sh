#!/bin/bash
# round 6: interleaved two-build headline A/B (old new old new new old): nobs-whisper_amd/lib/ab_old vs in-tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OLD=$PWD/nobs-whisper_amd/lib/ab_old/libwhisper_mi355x.so
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2 ${LAB_ARGS}"
for v in ${LAB_ORDER:-old new old new new old}; do
  if [ $v = old ]; then L=$OLD; else L=""; fi
  WHISPER_MI355X_LIB=$L timeout -k 10 300 python -u bench.py $X > gpurun_out/lab2_$v.json 2>/dev/null || { echo "$v FAIL"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/lab2_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', d['value'], d['extra']['phase_ms_last_step'], r['kernel'], r['avg_launch_ms'])"
done
