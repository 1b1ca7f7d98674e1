#!/bin/bash
# Round 3 closing pass (GPU box), each step under its own time limit, stopping at the first failure:
# the whole -m gpu suite, the default bench line (CPU baseline, variants incl. the serving line, app
# pattern, front-end), a rocprofv3 kernel-trace summary of the headline workload, the other BASELINE
# config lines and the strong-scaling shard sizes.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/rc_all.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/rc_all.log | tail -6; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench.py --variant-steps 2 --app-calls 4 > gpurun_out/rc_bench.json 2> gpurun_out/rc_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/rc_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/rc_bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_rc" -o run -- python3 "$R/bench.py" --cpu-baseline 0 --variants 0 --frontend 0 --app-pattern 0 > "$R/gpurun_out/prof_rc.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof_rc" "$R/gpurun_out/rc_kernels.md" | head -8
cd "$R"
bash tools/gpu_r03_cfg.sh
