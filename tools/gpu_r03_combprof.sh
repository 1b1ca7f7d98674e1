#!/bin/bash
# Round 3: rocprofv3 kernel summaries of the headline workload with 16 and 8 tokens per combine workgroup,
# same box (the env switch is read by the launcher; rocprofv3 runs python directly).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for t in 16 8; do
  WHISPER_MI355X_XCOMB_TOK=$t timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ct$t" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-baseline 0 --variants 0 --frontend 0 --app-pattern 0 > "$R/gpurun_out/prof_ct$t.log" 2>&1
  rc=$?; echo "tok $t rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 "$R/gpurun_out/prof_ct$t.log" | cut -c1-160
  python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof_ct$t" "$R/gpurun_out/ct${t}_kernels.md" > /dev/null
  grep -E "xattn_combine|xattn_qproj|xattn_step" "$R/gpurun_out/ct${t}_kernels.md"
done
