# cache-form cross step rows in flight per lane group: 8 vs 12 (WHISPER_MI355X_XSTEP_U12=1) at 16 / 32 clips
# (the WHISPER_MI355X_XSTEP_U12 variant was removed after this A/B: profiles/r05_xwide_ab.txt)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0 --app-pattern 0 --steps 3"
for cfg in "16 0" "16 1" "32 0" "32 1"; do
  set -- $cfg
  WHISPER_MI355X_XSTEP_U12=$2 timeout -k 10 300 python bench.py $X --global-batch $1 > gpurun_out/xu_$1_$2.json 2>/dev/null || { echo "$cfg FAIL"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/xu_$1_$2.json').read().strip().splitlines()[-1])
print('clips $1 u12 $2', d['value'], 'decode', d['extra']['phase_ms_last_step']['decode'])"
done
