"""Summarise a rocprofv3 SQLite database (kernel + memory-copy stats) as markdown.

Usage: python tools/rocpd_summary.py RUN_results.db [--per N] > profiles/x.md
``--per N`` divides totals by N (e.g. the number of fits in the run).
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    agg = {}
    for name, n, tot, avg, mx in rows:
        k = short(name)
        e = agg.setdefault(k, [0, 0.0, 0.0])
        e[0] += n
        e[1] += tot
        e[2] = max(e[2], mx)
    total = sum(v[1] for v in agg.values())
    print(f"## Kernels (per unit = total / {a.per:g})\n")
    print("| kernel | calls/unit | ms/unit | avg us | max us | % |")
    print("|---|---:|---:|---:|---:|---:|")
    for k, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"| `{k}` | {n / a.per:.1f} | {tot / 1e6 / a.per:.3f} | {tot / n / 1e3:.1f} | "
              f"{mx / 1e3:.1f} | {100 * tot / total:.1f} |")
    print(f"\nTotal kernel time per unit: {total / 1e6 / a.per:.3f} ms\n")
    try:
        mc = c.execute("select name, count(*), sum(duration), sum(size) from memory_copies "
                       "group by name order by sum(duration) desc").fetchall()
    except sqlite3.Error:
        mc = []
    if mc:
        print("## Memory copies\n")
        print("| direction | calls/unit | ms/unit | MB/unit |")
        print("|---|---:|---:|---:|")
        for name, n, tot, size in mc:
            print(f"| {name} | {n / a.per:.1f} | {tot / 1e6 / a.per:.3f} | "
                  f"{(size or 0) / 1e6 / a.per:.2f} |")


if __name__ == "__main__":
    main()
