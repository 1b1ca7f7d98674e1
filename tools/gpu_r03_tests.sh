#!/bin/bash
# Round-3 GPU pass: the new parity / error / batch-config tests, then (ALL=1) the whole -m gpu suite,
# then a short bench line and (AB="...") an env A/B of the bench (tools/gpu_envab.sh). Each step
# under its own time limit. Test failures (pytest rc 1) do not stop the later steps; a timeout, a
# crash or an abort (rc >= 2) ends the script there.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
fatal() { [ "$1" -ge 2 ] && [ "$1" -ne 5 ]; }
final=0
if [ "${NEW:-1}" = 1 ]; then
  timeout -k 10 ${T_NEW:-900} $T ${NEW_TESTS:-tests/test_gpu_errors.py tests/test_gpu_logits.py tests/test_gpu_batch_configs.py} -s > gpurun_out/r03_new.log 2>&1
  rc=$?; echo "new tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|max rel|prefixes|identical" gpurun_out/r03_new.log | cut -c1-300 | tail -40
  fatal $rc && exit $rc; [ $rc -eq 0 ] || final=$rc
fi
if [ "${ALL:-0}" = 1 ]; then
  timeout -k 10 900 $T -m gpu tests -q > gpurun_out/r03_all.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_all.log | tail -15
  fatal $rc && exit $rc; [ $rc -eq 0 ] || final=$rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --variant-steps 1 --app-calls 4 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
  rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/r03_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03_bench.err; exit $rc; }
fi
if [ -n "$AB" ]; then
  bash tools/gpu_envab.sh || exit $?
fi
if [ -n "$AB2" ]; then
  AB="$AB2" BENCH_ARGS="$BENCH_ARGS2" OUTP=envab2 bash tools/gpu_envab.sh || exit $?
fi
exit $final
