#!/bin/bash
# Round 3: key-split cache-form cross attention — the whole -m gpu suite, then same-box env A/Bs
# (XSPLIT=0 = one workgroup per (clip, head)) on the 16- and 32-clip shards and base f16 at 8 clips.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
if [ "${ALL:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/xs_all.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/xs_all.log | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
Q="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0"
for B in ${BATCHES:-16 32}; do
  AB="XSPLIT=0 base XSPLIT=0 base" OUTP=xs_b$B BENCH_ARGS="$Q --global-batch $B" bash tools/gpu_envab.sh || exit 1
done
