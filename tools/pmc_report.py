"""Per-kernel rocprofv3 PMC report (markdown) from one or more counter passes.

Usage: python tools/pmc_report.py --fits 2 DIR [DIR...]

Each DIR holds one ``rocprofv3 --pmc ... --output-format csv`` pass
(``*counter_collection.csv``; a pass run with ``--kernel-trace`` also leaves
``*kernel_trace.csv`` for durations). Counters are summed over every dispatch
of a kernel and divided by ``--fits`` (the traced program runs that many
identical fits), so per-level kernels report per-fit totals. Derived columns:

* VALU/wave, LDS/wave: SQ_INSTS_VALU / SQ_WAVES, SQ_INSTS_LDS / SQ_WAVES
* wait%, issue-stall%, active%: SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY
  as shares of SQ_WAVE_CYCLES (disjoint buckets on gfx950)
* LDS conflict%: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
* read / write MB: FETCH_SIZE / WRITE_SIZE KB / 1024 (FETCH_SIZE under-counts wide
  streams by up to 2x on gfx950 -- MI355X_MICROARCH.md); GB/s: their sum over the
  traced kernel time
"""

from __future__ import annotations

import argparse
import csv
import glob
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name).replace("void ", "")
    return name[:56]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--fits", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=16)
    a = ap.parse_args()
    ctr = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    dur = defaultdict(float)
    for d in a.dirs:
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(path) as fh:
                for r in csv.DictReader(fh):
                    k = short(r["Kernel_Name"])
                    ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    calls[k].add((d, r["Dispatch_Id"]))
        for path in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
            with open(path) as fh:
                for r in csv.DictReader(fh):
                    k = short(r["Kernel_Name"])
                    dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    f = a.fits
    rows = sorted(ctr, key=lambda k: -dur.get(k, 0.0))[: a.top]
    print("| kernel | calls/fit | us/fit | VALU/wave | LDS/wave | wait% | issue-stall% | active% "
          "| LDS conflict% | read MB/fit | write MB/fit | GB/s |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in rows:
        c = ctr[k]
        waves = c.get("SQ_WAVES", 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)

        def pct(name):
            return f"{100 * c[name] / wc:.0f}" if wc and name in c else ""

        per = (lambda n: f"{c[n] / waves:.0f}" if waves and n in c else "")
        lds = (f"{100 * c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.1f}"
               if c.get("SQ_LDS_IDX_ACTIVE") else "")
        rd = c.get("FETCH_SIZE", 0.0) / 1024 / f
        wr = c.get("WRITE_SIZE", 0.0) / 1024 / f
        mb = rd + wr
        us = dur.get(k, 0.0) / f
        gbs = f"{mb / 1e3 / (us / 1e6):.0f}" if us and mb else ""
        n = len({x for x in calls[k]}) / max(1, len(a.dirs)) / f
        print(f"| `{k}` | {n:.1f} | {us:.1f} | {per('SQ_INSTS_VALU')} | {per('SQ_INSTS_LDS')} | "
              f"{pct('SQ_WAIT_ANY')} | {pct('SQ_WAIT_INST_ANY')} | {pct('SQ_ACTIVE_INST_ANY')} | "
              f"{lds} | {rd:.1f} | {wr:.1f} | {gbs} |")


if __name__ == "__main__":
    main()
