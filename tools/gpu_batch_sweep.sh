cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for B in 16 32 64; do
  timeout -k 10 300 python3 bench.py --global-batch $B --steps 2 --warmup 1 --variants 0 --cpu-baseline 0 > gpurun_out/gb_$B.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/gb_$B.json').read().strip().splitlines()[-1]); print($B, d['value'], d['ms_per_step'], d['extra']['phase_ms_last_step'])"
done
