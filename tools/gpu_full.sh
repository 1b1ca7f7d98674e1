#!/bin/bash
# GPU box: PMC traffic passes of the roofline kernels -> profiles/<tag>_pmc_traffic.json (copied to
# gpurun_out/), then the full default bench (reads that file) and its rocprof kernel summary.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01e}"
cd "$R" && mkdir -p gpurun_out
bash tools/pmc.sh || exit 1
python3 tools/pmc_traffic.py "$TAG" && cp "profiles/${TAG}_pmc_traffic.json" gpurun_out/ || exit 1
bash tools/gpu_bench.sh
