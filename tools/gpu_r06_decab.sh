#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dec_gemm_ab.py > gpurun_out/r06_dec_gemm_ab.txt 2>&1; rc=$?
cat gpurun_out/r06_dec_gemm_ab.txt | grep -v amdgpu.ids
exit $rc
