#!/usr/bin/env python3
"""Per-kernel summary (calls, avg/total µs) from a rocprofv3 rocpd database (run_results.db).
    python tools/rocpd_summary.py gpurun_out/prof_dm/run_results.db [name-filter]"""
import sqlite3
import sys


def summary(db, filt=""):
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    q = (f"select s.kernel_name, count(*), avg(d.end-d.start)/1000.0, sum(d.end-d.start)/1000.0 from {kd} d "
         f"join {ks} s on d.kernel_id=s.id group by s.kernel_name order by sum(d.end-d.start) desc")
    return [r for r in c.execute(q) if filt in r[0]]


if __name__ == "__main__":
    for name, cnt, avg, tot in summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print(f"{avg:10.2f} us avg  x{cnt:5d}  {tot:10.1f} us total  {name[:100]}")
