#!/bin/bash
# Round 3 closing measurements (GPU box), each step under its own time limit, stopping at the first
# failure: PMC HBM-traffic passes for the 128/64/32/16-clip workloads (-> profiles/r03_pmc_traffic.json,
# which the bench then reads), MFMA-busy passes, the default bench line (with the CPU baseline), and a
# rocprofv3 kernel-trace summary of the same bench.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
BATCHES="${PMC_BATCHES:-128 64 32 16}" bash tools/pmc.sh || exit $?
python3 tools/pmc_traffic.py r03 | tail -12 || exit 1
bash tools/pmc_mfma.sh r03 || exit $?
cd "$R"
timeout -k 10 900 python -u bench.py > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/r03f_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03f_bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03f" -o run -- python3 "$R/bench.py" --cpu-baseline 0 --variants 0 --frontend 0 --app-pattern 0 > "$R/gpurun_out/prof_r03f.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$R/gpurun_out/prof_r03f.log"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof_r03f" "$R/gpurun_out/r03f_kernels.md" | head -24
