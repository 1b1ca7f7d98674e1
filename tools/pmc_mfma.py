"""MFMA-busy fraction per kernel from tools/pmc_mfma.sh's counter CSVs.

busy = SQ_VALU_MFMA_BUSY_CYCLES (MFMA pipe cycles summed over the SIMDs that ran the dispatch;
32 per 32x32x16 bf16 MFMA, MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units"); the dispatch's
clock cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs). MFMA-busy fraction =
busy / (cycles x 1024 SIMDs) (256 CUs x 4). Writes profiles/<tag>_pmc_mfma.json (tag: argv[1], default r02)
and the same file under gpurun_out/ (which travels back from the GPU box).
"""
import csv
import glob
import json
import sys
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read(d):
    acc = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = f'{row["Kernel_Name"]}@grid={row["Grid_Size"]}'
                c = acc[k][row["Counter_Name"]]
                c[0] += 1
                c[1] += float(row["Counter_Value"])
    return acc


def main():
    out = {}
    for tag in ("bf16", "fp8"):
        for k, cs in read(os.path.join(ROOT, "gpurun_out", f"pmc_mfma_{tag}")).items():
            nb, busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", (0, 0.0))
            ng, grbm = cs.get("GRBM_GUI_ACTIVE", (0, 0.0))
            if not nb or not ng:
                continue
            b, g = busy / nb, grbm / ng
            rec = dict(launches=nb, mfma_busy_cycles=b, grbm_gui_active=g, mfma_busy_frac=b / (g / 8.0 * 1024.0))
            # the stall counters (per dispatch; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles,
            # MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units"): shares of the waves' lifetime
            avg = {c: v / n for c, (n, v) in cs.items() if n}
            wc = avg.get("SQ_WAVE_CYCLES")
            if wc:
                for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                    if c in avg:
                        rec[c.lower() + "_share"] = avg[c] / wc
            if avg.get("SQ_LDS_IDX_ACTIVE"):
                rec["lds_bank_conflict_share"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]
            rec["counters"] = avg
            out[f"{tag}:{k}"] = rec
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_mfma.json")
    for p in (path, os.path.join(ROOT, "gpurun_out", f"{tag}_pmc_mfma.json")):
        with open(p, "w") as fh:
            json.dump(out, fh, indent=1)
    for k, v in out.items():
        extra = "  ".join(f"{c[:-6]} {v[c]:.3f}" for c in v if c.endswith("_share"))
        print(f"{v['mfma_busy_frac']:.3f} busy  n={v['launches']}  {extra}  {k[:100]}")
    print("wrote", path)


if __name__ == "__main__":
    main()
