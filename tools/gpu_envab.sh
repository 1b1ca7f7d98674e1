#!/bin/bash
# bench A/B of two environment settings on one box: AB_A="X=1" AB_B="Y=2" [BARGS=...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for v in A B A B; do
  eval envs=\$AB_$v
  timeout -k 10 400 env BENCH_KTIME=0 $envs python bench.py --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 ${BARGS} > gpurun_out/eab_$v.log 2> gpurun_out/eab_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 gpurun_out/eab_$v.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/eab_$v.log').read().strip().splitlines()[-1]); print('$v', '$envs', d['value'], d['extra']['phase_ms_last_step'])"
done
