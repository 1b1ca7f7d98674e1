#!/bin/bash
# rocprofv3 kernel trace of short bench runs at B = 128 and B = 16 -> decode-step timelines
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for B in ${BATCHES:-128 16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d "$R/gpurun_out/tl_$B" -o run -- \
    python3 "$R/bench.py" --global-batch $B --tokens 16 --steps 1 --warmup 1 --variants 0 --cpu-baseline 0 \
    > "$R/gpurun_out/tl_$B.log" 2>&1 || { echo "rocprof B=$B failed"; tail -5 "$R/gpurun_out/tl_$B.log"; exit 1; }
  python3 "$R/tools/timeline.py" "$R/gpurun_out/tl_$B" "$R/gpurun_out/timeline_b$B.md" | tail -30
  rm -rf "$R/gpurun_out/tl_$B"
done
