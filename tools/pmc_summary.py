"""Summarise rocprofv3 PMC CSV output per kernel (last dispatch of each kernel name).

Usage: python tools/pmc_summary.py DIR [DIR...]   (directories holding *counter_collection.csv)
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    rows = defaultdict(dict)
    for d in sys.argv[1:]:
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            last = {}
            with open(path) as fh:
                for r in csv.DictReader(fh):
                    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
                    key = (name, r["Counter_Name"])
                    disp = int(r["Dispatch_Id"])
                    prev = last.get(key)
                    if prev is None or disp > prev[0]:
                        last[key] = (disp, float(r["Counter_Value"]))
            for (name, cn), (_, v) in last.items():
                rows[name][cn] = v
    names = sorted({c for r in rows.values() for c in r})
    print("kernel".ljust(50) + "".join(c[:22].rjust(24) for c in names))
    for k, r in sorted(rows.items()):
        print(k.ljust(50) + "".join(f"{r.get(c, float('nan')):24.4g}" for c in names))


if __name__ == "__main__":
    main()
