cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for nt in 0 2 0 2; do
  NS=128 WHISPER_MI355X_XNT=$nt timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/xt$nt -o run -- python3 $R/tools/xattn_tune.py > $R/gpurun_out/xt$nt.log 2>&1 || exit 1
  echo "XNT=$nt"; python3 $R/tools/prof_summary.py $R/gpurun_out/xt$nt $R/gpurun_out/xt$nt.md | grep -E "xattn_step"
done
