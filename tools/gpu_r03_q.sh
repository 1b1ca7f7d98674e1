#!/bin/bash
# Round 3: quantized-file tests, then large-v3 f16 vs large-v3-q5_0 decode at 1 and 128 clips.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_quant.py > gpurun_out/r03q_tests.log 2>&1
rc=$?; echo "quant tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r03q_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
Q="--tokens 128 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0"
for spec in ${SPECS:-"none 128" "q5_0 128" "q5_0 1" "none 1"}; do
  set -- $spec
  timeout -k 10 600 python -u bench.py --dtype f16 --quant $1 --global-batch $2 --steps 1 --warmup 1 $Q \
      > gpurun_out/r03q_$1_$2.json 2> gpurun_out/r03q_$1_$2.err
  rc=$?; echo "quant $1 B=$2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03q_$1_$2.err; exit $rc; }
  python3 - gpurun_out/r03q_$1_$2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print(f"  {d['config']['workload'][:40]:40s} value {d['value']:9.1f}  phases {e['phase_ms_last_step']}  arena {e['weight_arena_bytes'] / 1e9:.3f} GB")
PY
done
