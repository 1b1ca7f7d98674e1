#!/bin/bash
# Round 3, pass F: the whole -m gpu suite, then the small-M threshold A/B at 4 and 8 clips (large-v3 bf16).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
if [ "${ALL:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03f_all.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r03f_all.log | tail -8
  [ $rc -le 1 ] || exit $rc
fi
for B in ${BS:-4 8}; do
  AB="SMALLM=0 SMALLM=$B SMALLM=0 SMALLM=$B" OUTP=absm$B \
    BENCH_ARGS="--global-batch $B --steps 3 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0" \
    bash tools/gpu_envab.sh || exit $?
done
