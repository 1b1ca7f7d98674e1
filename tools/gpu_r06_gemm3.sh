#!/bin/bash
# round 6: encoder GEMM epilogues: coalesced (default) vs transposed-accumulator direct stores (TR): bitwise A/B on
# the encoder shapes, kernel / encoder parity with TR, clock stamps of both, headline bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_dv_ab.py > gpurun_out/r06_gemm_tr_ab.txt 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/r06_gemm_tr_ab.txt; exit 1; }
cat gpurun_out/r06_gemm_tr_ab.txt
WHISPER_MI355X_GEMM_TR=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_parity.py \
    > gpurun_out/r06_gemm3_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r06_gemm3_tests.txt; exit 1; }
tail -2 gpurun_out/r06_gemm3_tests.txt
for v in -1 14; do
  timeout -k 10 200 python -u tools/gemm_stamps.py $v > gpurun_out/r06_gemm_stamps_v$v.txt 2>&1 || { echo "stamps rc=$?"; tail -5 gpurun_out/r06_gemm_stamps_v$v.txt; exit 1; }
  cat gpurun_out/r06_gemm_stamps_v$v.txt
done
BENCH_ARGS="--steps 4 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0" \
  AB="base GEMM_TR=1 base GEMM_TR=1" OUTP=r06_trab bash tools/gpu_envab.sh
