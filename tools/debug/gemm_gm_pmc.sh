# FETCH_SIZE per encoder GEMM launch for two tile orders (WHISPER_MI355X_GEMM_GM = 0 / 4), counters only
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
ARGS="--tokens 4 --steps 1 --warmup 1 --cpu-baseline 0 --variants 0 --frontend 0 --app-pattern 0 --f16-line 0"
for gm in 0 4; do
  d="$R/gpurun_out/pmc_gm$gm"
  WHISPER_MI355X_GEMM_GM=$gm timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemm8p_kernel" --output-format csv -d "$d" -o run \
      -- python3 "$R/bench.py" $ARGS > "$d.log" 2>&1
  rc=$?; echo "gm=$gm rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$d.log"; exit $rc; }
  python3 - "$d" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: [0, 0.0])
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") == "FETCH_SIZE":
            k = r["Kernel_Name"][:70] + " grid=" + r["Grid_Size"]
            acc[k][0] += 1; acc[k][1] += float(r["Counter_Value"])
for k, (n, v) in sorted(acc.items()):
    print(f"  {2 * v * 1024 / n / 1e6:9.1f} MB fetch/launch (x2 gfx950)  n={n}  {k}")
PY
done
