"""Decode-step timeline from a rocprofv3 --kernel-trace result (SQLite .db): for the last decode
step of the run (the dispatches between the last two logits_kernel launches), each kernel in
order with its duration and the idle gap before it, then per-kernel-name sums over the step.
Usage: python tools/timeline.py <dir with *.db> [out.md]"""
import glob
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void wm::", "").replace("wm::", "")
    return re.sub(r"<.*", "", name)[:40]


def main():
    dbs = glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True)
    rows = []
    for db in dbs:
        con = sqlite3.connect(db)
        rows += con.execute("""select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
                               join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
    rows.sort(key=lambda r: r[1])
    idx = [i for i, r in enumerate(rows) if "logits_kernel" in r[0]]
    a, b = idx[-2] + 1, idx[-1] + 1
    step = rows[a:b]
    out = [f"decode step: {len(step)} kernels, {(step[-1][2] - step[0][1]) / 1e3:.1f} us first start -> last end", "",
           "| # | kernel | us | gap before us |", "|---|---|---|---|"]
    agg = {}
    prev_end = rows[a - 1][2]
    for i, (n, s, e) in enumerate(step):
        k = short(n)
        c, t, g = agg.get(k, (0, 0.0, 0.0))
        agg[k] = (c + 1, t + (e - s) / 1e3, g + (s - prev_end) / 1e3)
        if i < 40:
            out.append(f"| {i} | {k} | {(e - s) / 1e3:.2f} | {(s - prev_end) / 1e3:.2f} |")
        prev_end = e
    out += ["", "| kernel | calls | sum us | avg us | sum of gaps before |", "|---|---|---|---|---|"]
    for k, (c, t, g) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append(f"| {k} | {c} | {t:.1f} | {t / c:.2f} | {g:.1f} |")
    tot = sum(v[1] for v in agg.values())
    gaps = sum(v[2] for v in agg.values())
    out.append(f"| **total** | {len(step)} | {tot:.1f} | | {gaps:.1f} |")
    txt = "\n".join(out)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
