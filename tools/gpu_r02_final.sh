#!/bin/bash
# Round-2 closing pass (GPU box): GPU test suite, smoke, default bench line (CPU baseline, variants,
# front-end), rocprofv3 kernel summary of a short bench, then the secondary BASELINE config lines.
# Each step has its own time limit; a failure ends the run. Outputs under gpurun_out/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; }
step tests && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f_tests.log; [ $rc -eq 0 ] || exit $rc
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/f_smoke.log; [ $rc -eq 0 ] || exit $rc
step bench && timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err
rc=$?; tail -c 300 gpurun_out/f_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/f_bench.err; exit $rc; }
step prof && BENCH_ARGS="--tokens 32 --steps 1 --warmup 1 --cpu-baseline 0 --variants 0 --frontend 0" bash tools/gpu_prof.sh || exit $?
cd "$R"
run() {
  local tag=$1; shift
  timeout -k 10 600 python3 bench.py --variants 0 --frontend 0 "$@" > "gpurun_out/f_cfg_$tag.json" 2> "gpurun_out/f_cfg_$tag.err"
  local rc=$?; echo "$tag rc=$rc"; tail -c 200 "gpurun_out/f_cfg_$tag.json"; return $rc
}
step cfg && run base_f16_b1 --model base --dtype f16 --batch 1 --steps 3 --warmup 1 &&
run small_bf16_b32 --model small --batch 32 --steps 2 --warmup 1 &&
run turbo_bf16_b256 --model large-v3-turbo --batch 256 --steps 2 --warmup 1 --cpu-baseline 0 &&
run turbo_fp8_b256 --model large-v3-turbo --dtype fp8 --batch 256 --steps 2 --warmup 1 --cpu-baseline 0 &&
run largev3_b16 --global-batch 16 --steps 2 --warmup 1 --cpu-baseline 0
