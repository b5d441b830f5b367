"""Print the kernel / copy timeline of the last fit in a rocprofv3 database.

Usage: python tools/rocpd_timeline.py RUN_results.db [--first-kernel edges_kernel] [--n 80]
Shows each dispatch's start offset, duration and the idle gap before it (us):
gaps are host-side overhead the GPU waited through.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first-kernel", default="edges_kernel")
    ap.add_argument("--n", type=int, default=80)
    ap.add_argument("--agg", action="store_true",
                    help="per-kernel totals of the last fit instead of the timeline")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.first_kernel in r[0]]
    if not idx:
        raise SystemExit("marker kernel not found")
    fit = rows[idx[-1]:]
    t0 = fit[0][1]
    if a.agg:
        tot = {}
        for name, st, en in fit:
            short = name.split("(")[0].replace("void ", "")[:60]
            cnt, d = tot.get(short, (0, 0.0))
            tot[short] = (cnt + 1, d + (en - st) / 1e3)
        span = (max(r[2] for r in fit) - t0) / 1e3
        print(f"last fit: span {span:.1f} us, kernel time {sum(d for _, d in tot.values()):.1f} us")
        print(f"{'kernel':62s} {'calls':>5s} {'total us':>9s} {'avg us':>7s}")
        for k, (cnt, d) in sorted(tot.items(), key=lambda x: -x[1][1]):
            print(f"{k:62s} {cnt:5d} {d:9.1f} {d / cnt:7.1f}")
        return
    prev = t0
    gaps = 0.0
    for k, (name, st, en) in enumerate(fit):
        gap = max(0.0, (st - prev) / 1e3)
        gaps += gap
        if k < a.n:
            short = name.split("(")[0].replace("void ", "")[:44]
            print(f"{short:46s} t={(st - t0) / 1e3:9.1f} dur={(en - st) / 1e3:8.1f} gap={gap:7.1f}")
        prev = max(prev, en)
    print(f"span {(prev - t0) / 1e3:.1f} us, idle gaps {gaps:.1f} us, kernels {len(fit)}")


if __name__ == "__main__":
    main()
