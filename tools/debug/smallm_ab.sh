# decode path A/B at the strong-scaling shard sizes: the split-K launch chain vs the small-M path (one-launch
# GEMMs with the LayerNorm prologue) for every decode step (WHISPER_MI355X_SMALLM=1: up to 32 clips)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
for B in 16 32; do
  for sm in 0 1 0 1; do
    WHISPER_MI355X_SMALLM=$([ $sm = 1 ] && echo 1 || echo 4) timeout -k 10 300 python bench.py $X --global-batch $B > gpurun_out/sm_$B_$sm.json 2>/dev/null || { echo "B=$B sm=$sm FAIL"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/sm_$B_$sm.json').read().strip().splitlines()[-1]); print('B=$B smallm_all=$sm', d['value'], d['extra']['phase_ms_last_step']['decode'])"
  done
done
