cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
DEC_M=128 DEC_SPLITS=${DEC_SPLITS:-0,1} timeout -k 10 300 python3 -u tools/dec_tune.py > gpurun_out/dec_tune.log 2>&1
rc=$?; cat gpurun_out/dec_tune.log; exit $rc
