"""Per-kernel summary of a rocprofv3 rocpd database: calls, total and mean us.

Usage: python tools/rocpd_top.py gpurun_out/prof_on/run_results.db [N]
"""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = sqlite3.connect(db)
q = ("select name, count(*), sum(end - start) / 1000.0 from kernels group by name "
     "order by sum(end - start) desc limit ?")
for name, calls, tot in c.execute(q, (top,)):
    print(f"{name[:70]:70s} {calls:6d} {tot:10.1f} us {tot / calls:9.1f} us/call")
