#!/bin/bash
# full GPU test suite, then a 16-clip A/B of the split rule
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t_tests.log; [ $rc -eq 0 ] || exit $rc
AB_A="WHISPER_MI355X_DEC_FILL=0" AB_B="X=0" BARGS="--global-batch 16" bash tools/gpu_envab.sh
