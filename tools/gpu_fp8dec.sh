#!/bin/bash
# fp8 decoder weights: kernel + end-to-end tests, then turbo fp8 B=256 and large-v3 fp8 B=128 A/B
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/fp8dec_tests.log 2>&1
rc=$?; grep -E "fp8 decoder|passed|failed|Error" gpurun_out/fp8dec_tests.log | tail -5; [ $rc -eq 0 ] || { tail -30 gpurun_out/fp8dec_tests.log; exit $rc; }
run() {
  timeout -k 10 500 env $3 python bench.py $2 --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 > gpurun_out/fp8d_$1.log 2> gpurun_out/fp8d_$1.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -5 gpurun_out/fp8d_$1.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/fp8d_$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['extra']['phase_ms_last_step'])"
}
run turbo_dec8 "--model large-v3-turbo --global-batch 256 --dtype fp8" "X=1" && \
run turbo_dec16 "--model large-v3-turbo --global-batch 256 --dtype fp8" "WHISPER_MI355X_FP8_DEC=0" && \

run lv3_dec8 "--dtype fp8" "X=1" && \
run lv3_dec16 "--dtype fp8" "WHISPER_MI355X_FP8_DEC=0"
