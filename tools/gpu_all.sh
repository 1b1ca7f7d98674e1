#!/bin/bash
# Round-2 full GPU pass: every -m gpu test, the smoke, the default bench (with the reference-workload
# variants and the CPU baseline), then the strong-scaling batch sweep (global batch 16/32/64).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export NW_MODEL_DIR=/tmp/nw_models
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_all.log; grep -E "FAIL|ERROR" gpurun_out/pytest_all.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err
rc=$?; tail -c 600 gpurun_out/bench_all.json; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_SWEEP" ] || bash tools/gpu_batch_sweep.sh
