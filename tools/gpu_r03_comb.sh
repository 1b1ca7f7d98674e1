#!/bin/bash
# Round 3: xattn_combine at 8 tokens per workgroup — bitwise switch tests + xattn kernel tests, then
# same-box env A/Bs (XCOMB_TOK=16 = the previous shape) at 128 and 64 clips.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch_configs.py::test_direct_form_switches_bit_identical tests/test_gpu_xattn.py > gpurun_out/comb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/comb_tests.log
[ $rc -eq 0 ] || exit $rc
Q="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0"
for B in ${BATCHES:-128 64}; do
  AB="${AB:-XCOMB_TOK=16 base XCOMB_TOK=16 base}" OUTP=comb_b$B BENCH_ARGS="$Q --global-batch $B" bash tools/gpu_envab.sh || exit 1
done
