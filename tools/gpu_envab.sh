#!/bin/bash
# Same-box A/B of engine env switches on the headline bench (short runs, no extras). Usage:
#   AB="XSERP=0 XSERP=1 XSERP=1,XNT=0" bash tools/gpu_envab.sh     (each token: comma-separated
#   WHISPER_MI355X_<NAME>=<value> pairs; "base" = no override). Output: gpurun_out/envab_<i>.json
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0}"
i=0
for spec in ${AB:-base}; do
  envs=()
  if [ "$spec" != base ]; then
    IFS=',' read -ra kv <<< "$spec"
    for x in "${kv[@]}"; do envs+=("WHISPER_MI355X_$x"); done
  fi
  timeout -k 10 ${T_AB:-300} env "${envs[@]}" python -u bench.py $ARGS > gpurun_out/${OUTP:-envab}_$i.json 2> gpurun_out/${OUTP:-envab}_$i.err
  rc=$?
  python3 - "$spec" gpurun_out/${OUTP:-envab}_$i.json <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"{sys.argv[1]:28s} value {d['value']:8.1f}  ms/step {d['ms_per_step']:8.1f}  phases {d['extra']['phase_ms_last_step']}  "
          f"{r['kernel']} {r['avg_launch_ms']*1e3:.1f} us frac {r['frac']}")
except Exception as e:
    print(sys.argv[1], "no result", e)
PY
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/${OUTP:-envab}_$i.err; exit $rc; }
  i=$((i+1))
done
