# decode FC1 (N >= 4096) split count: heuristic (3 for large-v3) vs WHISPER_MI355X_DEC_WIDE_SPLITS=1 / 2
# (the WHISPER_MI355X_DEC_WIDE_SPLITS knob was removed after this A/B: profiles/r05_fc1_splits_ab.txt)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0 --app-pattern 0 --steps 3"
for cfg in "128 0" "128 1" "128 2" "16 0" "16 1" "16 2"; do
  set -- $cfg
  WHISPER_MI355X_DEC_WIDE_SPLITS=$2 timeout -k 10 300 python bench.py $X --global-batch $1 > gpurun_out/ws_$1_$2.json 2>/dev/null || { echo "$cfg FAIL"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ws_$1_$2.json').read().strip().splitlines()[-1])
print('clips $1 wide_splits $2', d['value'], 'decode', d['extra']['phase_ms_last_step']['decode'])"
done
