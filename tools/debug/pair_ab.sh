# 128 clips as one batch vs two 64-clip halves in flight (WHISPER_MI355X_PAIR_MIN=64)
# (the WHISPER_MI355X_PAIR_MIN knob was removed after this A/B: profiles/r05_pair64_ab.txt)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0 --app-pattern 0 --steps 3"
for pm in 128 64; do
  WHISPER_MI355X_PAIR_MIN=$pm timeout -k 10 300 python bench.py $X > gpurun_out/pair_$pm.json 2>/dev/null || { echo "$pm FAIL"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/pair_$pm.json').read().strip().splitlines()[-1])
print('pair_min $pm', d['value'], d['extra']['phase_ms_last_step'])"
done
