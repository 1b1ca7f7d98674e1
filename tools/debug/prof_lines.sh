# rocprofv3 kernel stats of bench lines (tags and bench args in pairs; a tag old_* runs lib/ab_old's build)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
X="--variants 0 --cpu-baseline 0 --frontend 0 --f16-line 0 --inflight-line 0 --app-pattern 0"
while [ $# -ge 2 ]; do
  tag=$1; args=$2; shift 2
  lib=""; case $tag in old_*) lib=$PWD/nobs-whisper_amd/lib/ab_old/libwhisper_mi355x.so;; esac
  WHISPER_MI355X_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py $X $args > gpurun_out/prof_$tag.log 2>&1 || { echo "$tag FAIL"; exit 1; }
  rm -f gpurun_out/prof_$tag/run_kernel_trace.csv
  echo "== $tag: $(grep -c . gpurun_out/prof_$tag.log) log lines"
done
