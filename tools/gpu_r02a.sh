#!/bin/bash
# Round-2 check on the GPU box: the new parity tests (BASELINE config shapes, fallback decisions,
# long form, sizes-only context), the smoke, then a short default bench.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export NW_MODEL_DIR=/tmp/nw_models
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dist.py tests/test_gpu_configs.py > gpurun_out/pytest_r02a.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r02a.log; grep -E "PASS|FAIL|ERROR|SKIP" gpurun_out/pytest_r02a.log | tail -60 > gpurun_out/pytest_r02a_summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -4 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_r02a.json 2> gpurun_out/bench_r02a.err
rc=$?; tail -c 3000 gpurun_out/bench_r02a.json; tail -3 gpurun_out/bench_r02a.err; exit $rc
