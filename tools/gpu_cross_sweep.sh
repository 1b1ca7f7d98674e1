cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for B in 64 128; do for X in cache direct; do
  WHISPER_MI355X_CROSS=$X timeout -k 10 300 python3 bench.py --global-batch $B --steps 2 --warmup 1 --variants 0 --cpu-baseline 0 > gpurun_out/xs_${B}_$X.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/xs_${B}_$X.json').read().strip().splitlines()[-1]); print($B, '$X', d['value'], d['ms_per_step'], d['extra']['phase_ms_last_step'])"
done; done
