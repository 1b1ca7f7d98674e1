"""Per-launch HBM traffic from the two rocprofv3 --pmc passes of tools/pmc.sh.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch (TCC_EA0 request counters x 64 B). gfx950
correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly half the bytes of a wide coalesced
(16 B/lane) streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
Infinity-Cache hits are counted by these counters (not excluded).
Writes profiles/<tag>_pmc_traffic.json: {"<kernel symbol>@grid=<threads>": {launches, fetch_bytes,
write_bytes, traffic_bytes}} (per launch shape: e.g. the cross-attention kernel's prefill launches
cover several tokens per clip and must not be averaged with the decode-step launches).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read(counter: str, d: str):
    """d: a directory, or a glob of directories (one per workload: pmc_fetch_b128, pmc_fetch_b16, ...)"""
    acc = defaultdict(lambda: [0, 0.0])
    files = []
    for dd in sorted(glob.glob(d)):
        files += glob.glob(os.path.join(dd, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = f'{row["Kernel_Name"]}@grid={row["Grid_Size"]}'  # one entry per launch shape
                acc[k][0] += 1
                acc[k][1] += float(row["Counter_Value"])
    return acc


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    fetch = read("FETCH_SIZE", os.path.join(ROOT, "gpurun_out", "pmc_fetch*"))
    write = read("WRITE_SIZE", os.path.join(ROOT, "gpurun_out", "pmc_write*"))
    out = {}
    for k in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(k, (0, 0.0))
        nw, w = write.get(k, (0, 0.0))
        fb = 2.0 * f * 1024 / max(1, nf)
        wb = w * 1024 / max(1, nw)
        out[k] = dict(launches=max(nf, nw), fetch_bytes=fb, write_bytes=wb, traffic_bytes=fb + wb)
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_traffic.json")
    for p in (path, os.path.join(ROOT, "gpurun_out", f"{tag}_pmc_traffic.json")):  # gpurun_out travels back
        with open(p, "w") as fh:
            json.dump(out, fh, indent=1)
    for k, v in out.items():
        print(f"{v['traffic_bytes'] / 1e6:10.2f} MB/launch  (fetch x2 {v['fetch_bytes'] / 1e6:.2f}, write "
              f"{v['write_bytes'] / 1e6:.2f})  n={v['launches']}  {k[:90]}")
    print("wrote", path)


if __name__ == "__main__":
    main()
