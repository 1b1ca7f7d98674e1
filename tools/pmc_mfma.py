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
            out[f"{tag}:{k}"] = dict(launches=nb, mfma_busy_cycles=b, grbm_gui_active=g,
                                     mfma_busy_frac=b / (g / 8.0 * 1024.0))
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_mfma.json")
    for p in (path, os.path.join(ROOT, "gpurun_out", f"{tag}_pmc_mfma.json")):
        with open(p, "w") as fh:
            json.dump(out, fh, indent=1)
    for k, v in out.items():
        print(f"{v['mfma_busy_frac']:.3f} busy  n={v['launches']}  busy={v['mfma_busy_cycles']:.3e} "
              f"grbm={v['grbm_gui_active']:.3e}  {k[:110]}")
    print("wrote", path)


if __name__ == "__main__":
    main()
