#!/bin/bash
# compact GELU table: GPU test suite, then same-box library A/B (lib_ab/old.so = before, new.so = after)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/g_tests.log | head -20; exit $rc; }
bash tools/gpu_libab.sh
