#!/bin/bash
# round 6: the encoder's MFMA-busy and stall counter pass (r06_pmc_mfma.json), then a short headline bench with the
# new roofline fields (gemm_decode class, fp8 phase pricing checked on the turbo fp8 line)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_pipe.py \
    > gpurun_out/r06_pmc_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r06_pmc_tests.txt; exit 1; }
tail -2 gpurun_out/r06_pmc_tests.txt
bash tools/pmc_mfma.sh r06 > gpurun_out/r06_pmc_mfma.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/r06_pmc_mfma.log; exit 1; }
cat gpurun_out/r06_pmc_mfma.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --variants 0 --cpu-baseline 0 --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0 \
    > gpurun_out/r06_bench_quick.json 2> gpurun_out/r06_bench_quick.err || { echo "bench rc=$?"; tail -5 gpurun_out/r06_bench_quick.err; exit 1; }
tail -c 1500 gpurun_out/r06_bench_quick.json
timeout -k 10 300 python -u bench.py --model large-v3-turbo --dtype fp8 --global-batch 256 --steps 2 --warmup 1 --variants 0 --cpu-baseline 0 \
    --frontend 0 --app-pattern 0 --inflight-line 0 --f16-line 0 > gpurun_out/r06_turbo_fp8_quick.json 2> gpurun_out/r06_turbo_fp8_quick.err || { echo "fp8 bench rc=$?"; tail -5 gpurun_out/r06_turbo_fp8_quick.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r06_turbo_fp8_quick.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['phases']['encode'])"
