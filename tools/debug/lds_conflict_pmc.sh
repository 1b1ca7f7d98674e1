# LDS bank-conflict share of the LDS-DMA kernels of the headline step (one SQ pass, counters only)
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT}"
d="$R/gpurun_out/ldsc"
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS \
   --kernel-include-regex "gemm8p_kernel|xattn_step|attn_enc2|xattn_combine|gemm_dec_kernel" --output-format csv -d "$d" -o run \
   -- python3 "$R/bench.py" --tokens 4 --steps 1 --warmup 1 --cpu-baseline 0 --variants 0 --frontend 0 --app-pattern 0 --f16-line 0 --inflight-line 0 > "$d.log" 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$d.log"; exit $rc; }
python3 - "$d" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(acc.items()):
    w = v["SQ_WAVE_CYCLES"] or 1
    print("%-60s LDS conflict %5.1f %%  parked %5.1f %%  issue-stall %5.1f %%  issuing %5.1f %%" % (
        k, 100 * v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"]), 100 * v["SQ_WAIT_ANY"] / w,
        100 * v["SQ_WAIT_INST_ANY"] / w, 100 * v["SQ_ACTIVE_INST_ANY"] / w))
PY
