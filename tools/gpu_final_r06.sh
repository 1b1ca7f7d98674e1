#!/bin/bash
# Round-6 final measurements on one GPU box (each step time-limited; a failure ends the script):
# the default bench + its rocprofv3 kernel summary, the PMC traffic of the roofline kernels at 128 clips,
# then the BASELINE config lines (tools/gpu_cfg_r06.sh). Trace files are removed after summarising.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
bash tools/gpu_bench.sh > gpurun_out/final_bench.txt 2>&1 || { echo "bench FAIL"; exit 1; }
rm -f gpurun_out/prof/*kernel_trace* gpurun_out/prof/*.db
echo "bench done"
BATCHES=128 bash tools/pmc.sh > gpurun_out/final_pmc.txt 2>&1 || { echo "pmc FAIL"; exit 1; }
python3 tools/pmc_traffic.py r06 >> gpurun_out/final_pmc.txt 2>&1 || { echo "pmc summary FAIL"; exit 1; }
echo "pmc done"
bash tools/gpu_cfg_r06.sh > gpurun_out/final_cfg.txt 2>&1 || { echo "cfg FAIL"; exit 1; }
echo "cfg done"
