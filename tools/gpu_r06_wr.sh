#!/bin/bash
# round 6: whole-row stores for the row-major encoder GEMM outputs (WHISPER_MI355X_GEMM_WR): isolated shapes, bitwise
# logits against the previous build, headline A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for wr in 0 1; do
  WHISPER_MI355X_GEMM_WR=$wr timeout -k 10 300 python -u tools/debug/xkv_shape.py 2>&1 | grep -v amdgpu.ids || exit 1
done
cp tools/debug/ref/envlg_x16_r06pre.npy gpurun_out/envlg_pre.npy
WHISPER_MI355X_GEMM_WR=1 timeout -k 10 200 python -u tools/debug/env_logits.py x16wr 16 cache || exit 1
python tools/debug/env_logits.py --compare pre x16wr || exit 1
rm -f gpurun_out/envlg_pre.npy gpurun_out/envlg_x16wr.npy
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
BENCH_ARGS="$X" AB="base GEMM_WR=1 base GEMM_WR=1" OUTP=r06_wr bash tools/gpu_envab.sh || exit 1
