# SQ counters of the E pass (xattn_step_kernel) on the large-v3 decode shape (tools/xattn_tune.py, 128 clips, 2 splits)
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT}"
d="$R/gpurun_out/xs_pmc"
NS=128 SPLITS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES \
   --kernel-include-regex xattn_step --output-format csv -d "$d" -o run -- python3 "$R/tools/xattn_tune.py" > "$d.log" 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$d.log"; exit $rc; }
python3 - "$d" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: [0, 0.0])
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]][0] += 1; acc[r["Counter_Name"]][1] += float(r["Counter_Value"])
for k, (n, v) in sorted(acc.items()):
    print(f"{k:28s} {v / n:16.0f} per dispatch  (n={n})")
PY
