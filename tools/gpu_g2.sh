#!/bin/bash
# decode row groups A/B: one graph (baseline), one graph with two branches, two graphs on two streams
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
B=${B:-128}
run() {
  timeout -k 10 400 env BENCH_KTIME=0 $2 python bench.py --global-batch $B --steps 2 --warmup 1 --variants 0 --frontend 0 --cpu-baseline 0 > gpurun_out/g2_$1.log 2> gpurun_out/g2_$1.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -5 gpurun_out/g2_$1.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/g2_$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['extra']['phase_ms_last_step'])"
}
run base "X=0" && run br2 "WHISPER_MI355X_DEC_STREAMS=2" && run gr2 "WHISPER_MI355X_DEC_STREAMS=2 WHISPER_MI355X_DEC_GRAPHS2=1" && run base2 "X=0" && run gr2b "WHISPER_MI355X_DEC_STREAMS=2 WHISPER_MI355X_DEC_GRAPHS2=1"
