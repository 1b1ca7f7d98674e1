#!/bin/bash
# Round-6 final, part 1 (one GPU box; each step time-limited, a failure ends the script): the default bench
# with its CPU baseline + the rocprofv3 kernel summary of the same command, then the PMC traffic passes.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
bash tools/gpu_bench.sh > gpurun_out/final_bench.txt 2>&1 || { echo "bench FAIL"; tail -5 gpurun_out/final_bench.txt; exit 1; }
rm -f gpurun_out/prof/*kernel_trace* gpurun_out/prof/*.db
echo "bench done"; grep '"metric"' gpurun_out/final_bench.txt | cut -c1-300
BATCHES=128 bash tools/pmc.sh > gpurun_out/final_pmc.txt 2>&1 || { echo "pmc FAIL"; tail -5 gpurun_out/final_pmc.txt; exit 1; }
python3 tools/pmc_traffic.py r06 >> gpurun_out/final_pmc.txt 2>&1 || { echo "pmc summary FAIL"; exit 1; }
echo "pmc done"; tail -5 gpurun_out/final_pmc.txt
