#!/bin/bash
# combine tokens-per-workgroup A/B (xattn tests under both, kernel timing, bench) + reduce prefetch check
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
for tb in 16 8; do
  timeout -k 10 300 env WHISPER_MI355X_XCOMB_TB=$tb python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_xattn.py tests/test_gpu_kernels.py > gpurun_out/comb_tests_$tb.log 2>&1
  rc=$?; echo "tests tb=$tb rc=$rc"; tail -2 gpurun_out/comb_tests_$tb.log; [ $rc -eq 0 ] || exit $rc
  WHISPER_MI355X_XCOMB_TB=$tb NS=128,64,16 timeout -k 10 120 python tools/xattn_tune.py || exit 1
done
for tb in 16 8 16 8; do
  timeout -k 10 400 env WHISPER_MI355X_XCOMB_TB=$tb python bench.py --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 > gpurun_out/comb_b_$tb.log 2> gpurun_out/comb_b_$tb.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/comb_b_$tb.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/comb_b_$tb.log').read().strip().splitlines()[-1]); print('tb=$tb', d['value'], d['extra']['phase_ms_last_step'])"
done
