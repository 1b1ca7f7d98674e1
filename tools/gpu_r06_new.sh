#!/bin/bash
# round 6: the new / tightened parity tests (pipelined decoding, full-depth configs[2] and the 16-clip shard, the
# fp8 / bf16 gates), then the encoder GEMM DMA-placement A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_dv_ab.py > gpurun_out/r06_gemm_dv_ab.txt 2>&1
echo "gemm A/B rc=$?"; cat gpurun_out/r06_gemm_dv_ab.txt | tail -6
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_pipe.py tests/test_gpu_fulldepth.py "tests/test_gpu_batch_configs.py::test_turbo_fp8_b256_vs_oracle" \
    > gpurun_out/r06_newtests.txt 2>&1
rc=$?
grep -E "worst step|identical|decisions clip|passed|failed|Error|error" gpurun_out/r06_newtests.txt | tail -60
exit $rc
