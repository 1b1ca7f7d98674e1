#!/bin/bash
# round 6: reduce + LayerNorm with one barrier pair fewer: bitwise logits old vs new library, interleaved 16-clip A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OLD=$PWD/nobs-whisper_amd/lib/ab_old/libwhisper_mi355x.so
WHISPER_MI355X_LIB=$OLD timeout -k 10 200 python -u tools/debug/env_logits.py lo 16 cache || exit 1
timeout -k 10 200 python -u tools/debug/env_logits.py ln 16 cache || exit 1
python tools/debug/env_logits.py --compare lo ln || exit 1
rm -f gpurun_out/envlg_l*.npy
LAB_ARGS="--global-batch 16" LAB_ORDER="old new old new new old new old" bash tools/gpu_r06_libab2.sh
