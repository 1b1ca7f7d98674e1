#!/bin/bash
# GPU box A/B: bench under two env settings (same process image, back to back), then a rocprofv3
# kernel summary of the first setting. Usage: AB_ENV_A="X=1" AB_ENV_B="X=2" bash tools/gpu_ab.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---cpu-baseline 0}"
for v in A B A B; do
  eval envs=\$AB_ENV_$v
  timeout -k 10 600 env $envs python bench.py $ARGS > gpurun_out/ab_$v.log 2> gpurun_out/ab_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 gpurun_out/ab_$v.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', '$envs', d['value'], d['extra']['phase_ms_last_step'], d['roofline']['avg_launch_ms'])"
done
[ -n "$PROF" ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 env $AB_ENV_A rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --tokens 32 --steps 1 --warmup 1 --cpu-baseline 0 > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof" "$R/gpurun_out/prof_summary.md" | head -24
