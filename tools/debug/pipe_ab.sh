# pipelined greedy decoding A/B (WHISPER_MI355X_PIPE 0 / 1) on the BASELINE configs' bench lines
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0"
run() {
  local tag=$1; shift
  for pipe in 0 1; do
    WHISPER_MI355X_PIPE=$pipe timeout -k 10 300 python bench.py $X "$@" > gpurun_out/pipe_${tag}_$pipe.json 2>/dev/null || { echo "$tag pipe=$pipe FAIL"; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/pipe_${tag}_$pipe.json').read().strip().splitlines()[-1])
ap = d.get('app_pattern') or []
aps = ' '.join('%s %.1f ms' % (a['model'], a['state_pool']['median_ms']) for a in ap)
print('$tag pipe=$pipe', d['value'], 'decode', d['extra']['phase_ms_last_step']['decode'], aps)"
  done
}
run base_b1 --model base --dtype f16 --global-batch 1 --steps 3 --app-pattern 1 &&
run lv3_b1 --model large-v3 --dtype f16 --global-batch 1 --steps 2 --app-pattern 0 &&
run lv3_b128 --steps 2 --app-pattern 0 &&
run lv3_b16 --global-batch 16 --steps 2 --app-pattern 0
