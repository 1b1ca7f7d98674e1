#!/bin/bash
# round 6: two half-batches in flight at small shards (8 / 16 / 32 / 64 clips): the serving line's rate vs one batch
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
X="--variants 1 --variant-steps 2 --fallback-line 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 1 --steps 2"
for b in ${INFL_BATCHES:-8 16 32 64}; do
  timeout -k 10 300 python -u bench.py $X --global-batch $b > gpurun_out/r06_infl_b$b.json 2> gpurun_out/r06_infl_b$b.err || { echo "b$b rc=$?"; tail -5 gpurun_out/r06_infl_b$b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06_infl_b$b.json').read().strip().splitlines()[-1])
v=[x for x in d['variants'] if 'in flight' in x['workload']]
print($b, 'one batch', d['value'], d['ms_per_step'], '| two in flight', v[0]['value'] if v else None, v[0]['ms_per_batch'] if v else None)"
done
