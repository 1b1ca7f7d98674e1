#!/bin/bash
# One GPU pass (gpurun): selected tests, optionally the whole -m gpu suite, a bench line. Every step
# under its own time limit; a timeout / crash / abort (rc >= 2, except pytest's "no tests" 5) ends the
# script there, test failures (rc 1) do not.
#   TESTS="tests/x.py ..."  ALL=1  BENCH=1  BENCH_ARGS="..."  TAG=name
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
TAG="${TAG:-r04}"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
fatal() { [ "$1" -ge 2 ] && [ "$1" -ne 5 ]; }
final=0
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TESTS:-1500} $T $TESTS -s > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|worst|identical|passed|failed" gpurun_out/${TAG}_tests.log | cut -c1-400 | tail -60
  fatal $rc && exit $rc; [ $rc -eq 0 ] || final=$rc
fi
if [ "${ALL:-0}" = 1 ]; then
  timeout -k 10 ${T_ALL:-1100} $T -m gpu tests -q ${ALL_ARGS} > gpurun_out/${TAG}_all.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_all.log | tail -15
  fatal $rc && exit $rc; [ $rc -eq 0 ] || final=$rc
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 ${T_BENCH:-900} python -u bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --variant-steps 1 --app-calls 4} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; cut -c1-1500 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
fi
exit $final
