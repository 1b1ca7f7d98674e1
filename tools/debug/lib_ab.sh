# A/B of two builds: nobs-whisper_amd/lib/ab_old/libwhisper_mi355x.so (before) vs the in-tree library (after):
# bitwise teacher-forced logits (tools/debug/ab_logits.py) and bench lines given as arguments
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
OLD=$PWD/nobs-whisper_amd/lib/ab_old/libwhisper_mi355x.so
WHISPER_MI355X_LIB=$OLD timeout -k 10 200 python tools/debug/ab_logits.py old && timeout -k 10 200 python tools/debug/ab_logits.py new || exit 1
python3 -c "
import numpy as np; a=np.load('gpurun_out/ab_old.npy'); b=np.load('gpurun_out/ab_new.npy')
print('logits bitwise equal:', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'max |diff|', float(np.abs(a-b).max()))"
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0 --app-pattern 0"
for cfg in "$@"; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=""; fi
    WHISPER_MI355X_LIB=$L timeout -k 10 300 python bench.py $X $cfg > gpurun_out/lab_$v.json 2>/dev/null || { echo "$cfg $v FAIL"; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/lab_$v.json').read().strip().splitlines()[-1])
print('$cfg', '$v', d['value'], 'decode', d['extra']['phase_ms_last_step']['decode'])"
  done
done
