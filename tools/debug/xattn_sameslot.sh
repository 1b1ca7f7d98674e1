# E pass: the engine's E layout vs every clip on one (cache-resident) E, kernel times by rocprofv3 --stats
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT}"
for same in 0 1; do
  d="$R/gpurun_out/xs_same$same"
  SAMESLOT=$([ $same = 1 ] && echo 1) NS=128 SPLITS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$d" -o run -- python3 "$R/tools/xattn_tune.py" > "$d.log" 2>&1 || { tail -5 "$d.log"; exit 1; }
  echo "same=$same"; grep "E " "$d.log" | tail -1
  f=$(find "$d" -name "*kernel_stats.csv" | head -1); grep -i "xattn" "$f" | cut -c1-200
done
