#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 SQLite output (the default format):
python tools/dbstats.py <results.db> [top]"""
import re
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
c = sqlite3.connect(db)
print(f"{'kernel':72s} {'calls':>6s} {'avg_us':>9s} {'total_us':>10s} {'pct':>6s}")
for name, calls, tot, avg, pct in c.execute(f"select name,total_calls,total_duration,average,percentage from top_kernels limit {top}"):
    name = re.sub(r"\(anonymous namespace\)::", "", str(name))[:72]
    print(f"{name:72s} {calls:6d} {avg:9.2f} {tot:10.1f} {pct:6.2f}")
