# combine token rule A/B on bench lines: WHISPER_MI355X_XCOMB_TOK=8 (the old fixed choice) vs the rule
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0 --app-pattern 0"
run() {
  local tag=$1; shift
  for tok in 8 0; do
    WHISPER_MI355X_XCOMB_TOK=$tok timeout -k 10 300 python bench.py $X "$@" > gpurun_out/xc_${tag}_$tok.json 2>/dev/null || { echo "$tag tok=$tok FAIL"; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/xc_${tag}_$tok.json').read().strip().splitlines()[-1])
print('$tag tok=$tok', d['value'], 'decode', d['extra']['phase_ms_last_step']['decode'])"
  done
}
run lv3_b128 --steps 3 && run lv3_b16 --global-batch 16 --steps 3 && run lv3_b64 --global-batch 64 --steps 3
