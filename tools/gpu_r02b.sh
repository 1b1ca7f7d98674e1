#!/bin/bash
# Round-2: selected GPU tests (PYTEST_K), the smoke, then a short default bench (BENCH_ARGS).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export NW_MODEL_DIR=/tmp/nw_models
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$PYTEST_K" \
    > gpurun_out/pytest_r02b.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_r02b.log; grep -E "FAIL|ERROR" gpurun_out/pytest_r02b.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NO_SMOKE" ]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -4 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench_r02b.json 2> gpurun_out/bench_r02b.err
rc=$?; tail -c 4000 gpurun_out/bench_r02b.json; tail -3 gpurun_out/bench_r02b.err; exit $rc
