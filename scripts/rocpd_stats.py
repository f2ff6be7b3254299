"""Kernel statistics from a rocprofv3 SQLite database (the rocpd format rocprofv3 writes by
default): per kernel name, calls, total / average duration, share of GPU time.
usage: python scripts/rocpd_stats.py RESULTS.db [--csv OUT] [--top N]"""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
rows = list(c.execute(f"select {name_col}, start, end from kernels"))
agg = {}
for n, s, e in rows:
    a = agg.setdefault(n, [0, 0])
    a[0] += 1
    a[1] += e - s
tot = sum(a[1] for a in agg.values())
lines = ["name,calls,total_ns,avg_ns,percent"]
for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    lines.append(f'"{n}",{k},{t},{t / k:.1f},{100.0 * t / tot:.2f}')
print(f"kernels: {len(rows)} dispatches, {len(agg)} names, {tot / 1e6:.3f} ms GPU time")
for l in lines[1:top + 1]:
    print(l)
if "--csv" in sys.argv:
    open(sys.argv[sys.argv.index("--csv") + 1], "w").write("\n".join(lines) + "\n")
