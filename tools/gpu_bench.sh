#!/bin/bash
# GPU box: full default bench (with the CPU baseline leg), then a rocprofv3 kernel-trace summary of
# the same command (CPU leg off). Every GPU step has its own time limit; a failure ends the run.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" ${BENCH_ARGS} --cpu-baseline 0 > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$R/gpurun_out/prof.log"
[ $rc -eq 0 ] || exit $rc
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof" "$R/gpurun_out/prof_summary.md" | head -30
