#!/bin/bash
# Round 3, pass C: the whole -m gpu suite, the headline bench line, and the large-v3-q5_0 measurements
# (HBM footprint and decode ms against f16 at B = 1 and B = 128). Each GPU step under
# its own time limit; a test failure does not stop the later steps, a timeout or crash does.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
final=0
if [ "${ALL:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests -q > gpurun_out/r03c_all.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03c_all.log | tail -12
  [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || final=$rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --variant-steps 1 --app-calls 4 > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err
  rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/r03c_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03c_bench.err; exit $rc; }
fi
if [ "${QUANT:-1}" = 1 ]; then
  Q="--tokens 128 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0"
  for spec in "none 1" "q5_0 1" "none 128" "q5_0 128"; do
    set -- $spec
    timeout -k 10 900 python -u bench.py --dtype f16 --quant $1 --global-batch $2 --steps 1 --warmup 1 $Q \
        > gpurun_out/r03c_q_$1_$2.json 2> gpurun_out/r03c_q_$1_$2.err
    rc=$?; echo "quant $1 B=$2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03c_q_$1_$2.err; exit $rc; }
    python3 - gpurun_out/r03c_q_$1_$2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print(f"  {d['config']['workload'][:40]:40s} value {d['value']:9.1f}  phases {e['phase_ms_last_step']}  arena {e['weight_arena_bytes'] / 1e9:.3f} GB")
PY
  done
fi
exit $final
