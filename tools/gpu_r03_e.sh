#!/bin/bash
# Round 3, pass E: the whole -m gpu suite on the working build, then a same-box A/B of library builds
# (nobs-whisper_amd/lib_ab/<v>.so, VERS order) on the 16-clip shard and on the 128-clip headline.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
if [ "${ALL:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03e_all.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r03e_all.log | tail -8
  [ $rc -le 1 ] || exit $rc
fi
Q="--variants 0 --frontend 0 --cpu-baseline 0 --app-pattern 0"
for B in ${BATCHES:-16 128}; do
  for v in ${VERS:-old mid new old mid new}; do
    timeout -k 10 300 env WHISPER_MI355X_LIB=$R/nobs-whisper_amd/lib_ab/$v.so python -u bench.py --global-batch $B --steps ${STEPS:-3} --warmup 1 $Q $MODEL_ARGS \
      > gpurun_out/lab_${B}_$v.json 2> gpurun_out/lab_${B}_$v.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $B $v rc=$rc"; tail -5 gpurun_out/lab_${B}_$v.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/lab_${B}_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('B=$B', '$v'.ljust(5), d['value'], d['extra']['phase_ms_last_step'], r['kernel'], round(r['avg_launch_ms']*1e3, 1))"
  done
done
