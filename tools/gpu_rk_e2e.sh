#!/bin/bash
# slab-free decode GEMMs end to end: GPU parity suite, then bench A/B (WHISPER_MI355X_DEC_RK=0 vs 1)
# at 16 clips (an 8-GPU strong-scaling shard) and 128 clips (the headline).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/e2e_tests.log 2>&1
rc=$?; tail -4 gpurun_out/e2e_tests.log; [ $rc -eq 0 ] || exit $rc
for B in 16 128; do
  for v in 0 1 0 1; do
    timeout -k 10 400 env WHISPER_MI355X_DEC_RK=$v python bench.py --global-batch $B --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 > gpurun_out/rk_b${B}_$v.log 2> gpurun_out/rk_b${B}_$v.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench B=$B rk=$v rc=$rc"; tail -5 gpurun_out/rk_b${B}_$v.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rk_b${B}_$v.log').read().strip().splitlines()[-1]); print('B=$B rk=$v', d['value'], d['extra']['phase_ms_last_step'])"
  done
done
