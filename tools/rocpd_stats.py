"""Per-kernel stats (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite db.

    python tools/rocpd_stats.py gpurun_out/<dir>/run_results.db > profiles/<name>_kernel_stats.csv
"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else "kernel_name"
rows = db.execute(f"select {name_col}, start, end from kernels").fetchall()
agg = {}
for name, s, e in rows:
    d = agg.setdefault(name, [])
    d.append(e - s)
tot_all = sum(sum(v) for v in agg.values())
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    t = sum(v)
    print(f'"{name}",{len(v)},{t},{t / len(v):.1f},{100.0 * t / tot_all:.4f},{min(v)},{max(v)}')
