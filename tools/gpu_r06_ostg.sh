#!/bin/bash
# round 6: E-pass partial-O stores staged through LDS (WHISPER_MI355X_XSTEP_OSTG): bitwise logits (40 clips, direct
# form), headline A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/debug/env_logits.py o0 40 direct || exit 1
WHISPER_MI355X_XSTEP_OSTG=1 timeout -k 10 200 python -u tools/debug/env_logits.py o1 40 direct || exit 1
python tools/debug/env_logits.py --compare o0 o1 || exit 1
rm -f gpurun_out/envlg_o*.npy
X="--variants 0 --cpu-baseline 0 --app-pattern 0 --frontend 0 --f16-line 0 --inflight-line 0 --steps 2"
BENCH_ARGS="$X" AB="${OSTG_AB:-base XSTEP_OSTG=1 base XSTEP_OSTG=1}" OUTP=r06_ostg bash tools/gpu_envab.sh
