#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite database (kernel time per symbol).

    python tools/rocpd_summary.py gpurun_out/prof/x/x_results.db [--top 20] [--md]
"""
import argparse
import sqlite3


def summary(path, top=20):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(
        f"select {name_col}, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
        f"from kernels group by {name_col} order by sum(end - start) desc limit ?", (top,)).fetchall()
    total = db.execute("select sum(end - start) from kernels").fetchone()[0] or 1
    return rows, total


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--top", type=int, default=20)
    p.add_argument("--md", action="store_true")
    a = p.parse_args()
    rows, total = summary(a.db, a.top)
    if a.md:
        print("| kernel | calls | total ms | avg us | min us | max us | % |")
        print("|---|---:|---:|---:|---:|---:|---:|")
    for name, n, tot, avg, mn, mx in rows:
        short = (name[:90] + "…") if len(name) > 90 else name
        if a.md:
            print(f"| `{short}` | {n} | {tot / 1e6:.3f} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {100 * tot / total:.1f} |")
        else:
            print(f"{n:6d} {tot / 1e6:10.3f} ms {avg / 1e3:10.1f} us {100 * tot / total:5.1f}%  {short}")


if __name__ == "__main__":
    main()
