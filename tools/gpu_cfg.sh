#!/bin/bash
# Bench lines of several configs in one GPU call: CFGS="name|bench args;name|bench args;..." (each under its
# own time limit; stops at the first failure)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
IFS=';' read -ra C <<< "$CFGS"
for c in "${C[@]}"; do
  name="${c%%|*}"; args="${c#*|}"
  timeout -k 10 ${T_CFG:-400} python -u bench.py $args > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err
  rc=$?; echo "cfg $name rc=$rc"
  python3 - "$name" <<'PY'
import json, sys
n = sys.argv[1]
try:
    d = json.load(open(f"gpurun_out/cfg_{n}.json"))
except Exception as e:
    print(n, "no json", e); sys.exit(0)
r = d["roofline"]
print(n, "value", d["value"], "ms/step", d["ms_per_step"], "phases", d["extra"]["phase_ms_last_step"],
      r["kernel"], "avg_ms", r["avg_launch_ms"], "frac", r["frac"])
for a in d.get("app_pattern") or []:
    print("  app", a.get("model"), a.get("state_pool"), a.get("no_pool"))
PY
  [ $rc -eq 0 ] || { tail -5 gpurun_out/cfg_$name.err; exit $rc; }
done
