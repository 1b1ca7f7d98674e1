#!/bin/bash
# GPU box: the default bench (headline, with the CPU baseline leg) + its rocprofv3 kernel summary,
# then large-v3 in the fp8 encoder mode (extra line). Each step has its own limit; failures end it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
bash tools/gpu_bench.sh || exit $?
cd "$R"
timeout -k 10 600 python bench.py --dtype fp8 --cpu-baseline 0 > gpurun_out/cfg_largev3_fp8_b128.json 2> gpurun_out/cfg_largev3_fp8_b128.err
rc=$?; echo "large-v3 fp8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('gpurun_out/cfg_largev3_fp8_b128.json')); print(d['value'], d['extra']['phase_ms_last_step'])"
