#!/bin/bash
# Round 3: XQ_FUSED rework — its bitwise test + the xattn kernel tests, then a same-box env A/B at 128 clips.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch_configs.py::test_xq_fused_equals_reduce_then_qproj tests/test_gpu_xattn.py > gpurun_out/xq_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/xq_tests.log
[ $rc -eq 0 ] || exit $rc
AB="XQ_FUSED=0 XQ_FUSED=1 XQ_FUSED=0 XQ_FUSED=1" OUTP=xqab bash tools/gpu_envab.sh
