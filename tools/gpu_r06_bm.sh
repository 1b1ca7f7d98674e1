#!/bin/bash
# round 6: decode GEMM row tile (isolated shapes + bitwise check, GEMM tests, bench lines)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r06_dec_bm_ab.txt
for cfg in ${BM_CFGS:-128,0 32,0}; do
  bm=${cfg%,*}; m64=${cfg#*,}
  WHISPER_MI355X_DEC_BM=$bm WHISPER_MI355X_DEC_M64=$m64 timeout -k 10 300 python -u tools/dec_bm_ab.py gpurun_out/bm_${bm}_${m64}.npz 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_dec_bm_ab.txt || exit 1
  python tools/dec_bm_ab.py --compare gpurun_out/bm_128_0.npz gpurun_out/bm_${bm}_${m64}.npz | tee -a gpurun_out/r06_dec_bm_ab.txt || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > gpurun_out/r06_bm_tests.txt 2>&1 || { tail -20 gpurun_out/r06_bm_tests.txt; exit 1; }
tail -2 gpurun_out/r06_bm_tests.txt
rm -f gpurun_out/bm_*.npz
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
for b in ${BM_BATCHES:-64 32 16}; do
  BENCH_ARGS="$X --global-batch $b" AB="${BM_AB:-DEC_BM=128 base DEC_BM=128 base}" OUTP=r06_bm_b$b bash tools/gpu_envab.sh || exit 1
done
