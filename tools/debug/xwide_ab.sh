# cache-form cross attention: 1024-thread kernel up to WHISPER_MI355X_XWIDE_MAX clips (default 4) on bench lines
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0 --app-pattern 0 --steps 3"
for cfg in "16 4" "16 16" "32 4" "32 32" "8 4" "8 8"; do
  set -- $cfg
  WHISPER_MI355X_XWIDE_MAX=$2 timeout -k 10 300 python bench.py $X --global-batch $1 > gpurun_out/xw_$1_$2.json 2>/dev/null || { echo "$cfg FAIL"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/xw_$1_$2.json').read().strip().splitlines()[-1])
print('clips $1 xwide_max $2', d['value'], 'decode', d['extra']['phase_ms_last_step']['decode'])"
done
