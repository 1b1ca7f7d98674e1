#!/bin/bash
# rocprofv3 kernel trace of a short bench run (GPU box): per-kernel summary -> gpurun_out/prof_summary.md
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---tokens 32 --steps 1 --warmup 1 --cpu-baseline 0}"
timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$R/gpurun_out/prof.log"
[ $rc -eq 0 ] || exit $rc
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof" "$R/gpurun_out/prof_summary.md" | head -40
