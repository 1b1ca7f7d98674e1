#!/bin/bash
# round 6: the whole GPU suite on the current build, then the smoke (each under its own limit)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -s > gpurun_out/r06_gputests_all.txt 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r06_gputests_all.txt | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06_gputests_all.txt | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/r06_smoke.txt; exit 1; }
tail -3 gpurun_out/r06_smoke.txt
