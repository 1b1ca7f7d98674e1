"""Summarise a rocprofv3 --kernel-trace result (SQLite .db or kernel_stats.csv) per kernel:
calls, total ms, average us, share. Usage: python tools/prof_summary.py <run_results.db|dir> [out.md]"""
import glob
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name.replace("void wm::", "").replace("wm::", "")[:90]


def from_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    rows = cur.execute("""select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
                          join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
    agg = {}
    for name, a, b in rows:
        n = short(name)
        c, t = agg.get(n, (0, 0.0))
        agg[n] = (c + 1, t + (b - a) * 1e-6)
    return agg


def main():
    src = sys.argv[1]
    if os.path.isdir(src):
        dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        src = dbs[0]
    agg = from_db(src)
    tot = sum(t for _, t in agg.values())
    lines = ["| kernel | calls | total ms | avg us | share |", "|---|---|---|---|---|"]
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| {n} | {c} | {t:.2f} | {1e3 * t / c:.2f} | {100 * t / tot:.1f}% |")
    lines.append(f"| **total** | {sum(c for c, _ in agg.values())} | {tot:.2f} | | |")
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
