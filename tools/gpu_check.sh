#!/bin/bash
# One GPU-box session: GPU tests, then (only if nothing faulted) a small bench and a rocprofv3
# kernel-trace summary. Every GPU step has its own time limit; a fault/abort/timeout ends the run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
[ -n "$BENCH_ARGS" ] || exit 0
timeout -k 10 ${T_BENCH:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
[ -n "$PROF" ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${T_BENCH:-600} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $BENCH_ARGS --cpu-baseline 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
exit $rc
