#!/bin/bash
# same-box A/B of two library builds (nobs-whisper_amd/lib_ab/old.so vs new.so) on the default bench
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for v in old new old new; do
  timeout -k 10 400 env WHISPER_MI355X_LIB=$R/nobs-whisper_amd/lib_ab/$v.so $ABENV python bench.py --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 ${BARGS} > gpurun_out/lab_$v.log 2> gpurun_out/lab_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 gpurun_out/lab_$v.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/lab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['extra']['phase_ms_last_step'])"
done
