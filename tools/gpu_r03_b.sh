#!/bin/bash
# Round 3, pass B: encoder attention variant tests + timing, a 128-clip env A/B, and a rocprofv3
# kernel-trace summary of the headline bench. Each GPU step under its own time limit; a timeout or a
# crash ends the script.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TESTS:-400} python -u -m pytest -v -s --timeout 200 --timeout-method thread $TESTS > gpurun_out/r03b_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|TF/s|assert" gpurun_out/r03b_tests.log | cut -c1-250 | tail -30
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$AB" ]; then
  bash tools/gpu_envab.sh || exit $?
fi
if [ "${PROF:-0}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r03 -- python3 -u bench.py --steps 2 --warmup 1 \
      --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 > gpurun_out/r03_prof_bench.json 2> gpurun_out/r03_prof_bench.err
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03_prof_bench.err; exit $rc; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
