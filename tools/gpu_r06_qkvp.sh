#!/bin/bash
# round 6: prefill QKV epilogue (EPI_QKV_DEC) on the whole-row map: bitwise prompted logits, old vs new library, then
# the prompted bench variants
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OLD=$PWD/nobs-whisper_amd/lib/ab_old/libwhisper_mi355x.so
for cfg in "16 cache" "40 direct"; do
  set -- $cfg
  WHISPER_MI355X_LIB=$OLD timeout -k 10 200 python -u tools/debug/env_logits.py old$1 $1 $2 prompt || exit 1
  timeout -k 10 200 python -u tools/debug/env_logits.py new$1 $1 $2 prompt || exit 1
  python tools/debug/env_logits.py --compare old$1 new$1 || exit 1
done
rm -f gpurun_out/envlg_*.npy
V="--variants 1 --variant-steps 2 --fallback-line 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 1"
for v in old new; do
  if [ $v = old ]; then L=$OLD; else L=""; fi
  WHISPER_MI355X_LIB=$L timeout -k 10 400 python -u bench.py $V > gpurun_out/r06_qkvp_$v.json 2> gpurun_out/r06_qkvp_$v.err || { tail -3 gpurun_out/r06_qkvp_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06_qkvp_$v.json').read().strip().splitlines()[-1])
print('$v headline', d['value'], d['extra']['phase_ms_last_step'])
for x in d['variants'][:3]: print('$v', x['workload'][:40], x['value'], x.get('phase_ms_last_step'))"
done
