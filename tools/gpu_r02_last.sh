#!/bin/bash
# last check of the round: GPU test suite, smoke, default bench line
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/l_tests.log 2>&1
rc=$?; tail -2 gpurun_out/l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/l_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/l_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/l_bench.json 2> gpurun_out/l_bench.err
rc=$?; tail -c 200 gpurun_out/l_bench.json; exit $rc
