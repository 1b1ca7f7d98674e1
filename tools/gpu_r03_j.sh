#!/bin/bash
# Round 3, pass J: whole -m gpu suite; A/B of the 1024-thread cache-form cross step at 1 and 4 clips;
# rocprofv3 kernel summary of base f16 at one clip (BASELINE configs[1]).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03j_all.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r03j_all.log | tail -6; [ $rc -le 1 ] || exit $rc
X="--variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0"
AB="XWIDE_MAX=0 base XWIDE_MAX=0 base" OUTP=abxw BENCH_ARGS="--model base --dtype f16 --global-batch 1 --steps 10 --warmup 2 $X" bash tools/gpu_envab.sh || exit $?
AB="XWIDE_MAX=0 base" OUTP=abxwl BENCH_ARGS="--global-batch 1 --steps 2 --warmup 1 $X" bash tools/gpu_envab.sh || exit $?
AB="XWIDE_MAX=0 base" OUTP=abxw4 BENCH_ARGS="--global-batch 4 --steps 2 --warmup 1 $X" bash tools/gpu_envab.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_b1" -o run -- python3 "$R/bench.py" --model base --dtype f16 --global-batch 1 --steps 5 --warmup 1 $X > "$R/gpurun_out/prof_b1.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof_b1" "$R/gpurun_out/b1_kernels.md" | head -24
