# xattn_combine tokens per workgroup (WHISPER_MI355X_XCOMB_TOK 8 / 16; _CV=1: Wv loaded before the partial sums): per-shape kernel times from the
# rocprofv3 trace of tools/xattn_tune.py and a hash of the output (equal hashes = the same bits)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp
for cfg in "8 0" "16 0" "16 1"; do
  set -- $cfg; tok=$1
  tag=xt$1_$2
  WHISPER_MI355X_XCOMB_CV=$2 WHISPER_MI355X_XCOMB_TOK=$tok NS=128,64,16 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/xattn_tune.py > gpurun_out/$tag.txt 2>&1 || { echo "$tag FAIL"; exit 1; }
  echo "tok=$tok cv=$2"; grep -h "^n=" gpurun_out/$tag.txt
  python3 - gpurun_out/$tag/run_kernel_trace.csv <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "xattn" in r["Kernel_Name"]:
        d[(r["Kernel_Name"][8:30], r["Grid_Size_X"], r["Grid_Size_Y"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items(): print("  ", k, len(v), "median %.2f us" % sorted(v)[len(v) // 2])
PY
done
