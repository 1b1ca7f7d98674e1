cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_xattn.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_xattn.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_xattn.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for pf in 0; do
  NS=128 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/xt$pf -o run -- python3 $R/tools/xattn_tune.py > $R/gpurun_out/xt$pf.log 2>&1 || exit 1
  grep "n=" $R/gpurun_out/xt$pf.log
  python3 $R/tools/prof_summary.py $R/gpurun_out/xt$pf $R/gpurun_out/xt$pf.md | grep -E "xattn"
done
