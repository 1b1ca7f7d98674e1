#!/bin/bash
# round 6: end-to-end bitwise checks of the switches that must not change bits (self-step heads per workgroup,
# decode GEMM row tile): teacher-forced logits of 16- and 40-clip batches, each setting in its own process
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 200 env "$@" || exit 1; }
run python -u tools/debug/env_logits.py b16 16 cache
run WHISPER_MI355X_SELF_HPB=4 python -u tools/debug/env_logits.py b16_hpb4 16 cache
run WHISPER_MI355X_DEC_BM=128 python -u tools/debug/env_logits.py b16_bm128 16 cache
run python -u tools/debug/env_logits.py b40 40 direct
run WHISPER_MI355X_SELF_HPB=1 WHISPER_MI355X_DEC_BM=128 python -u tools/debug/env_logits.py b40_alt 40 direct
python tools/debug/env_logits.py --compare b16 b16_hpb4 && python tools/debug/env_logits.py --compare b16 b16_bm128 &&
python tools/debug/env_logits.py --compare b40 b40_alt
