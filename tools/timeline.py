#!/usr/bin/env python3
"""Print a rocprofv3 kernel_trace.csv as a timeline (us from the first kernel):
queue, stream, start, end, duration, name; optional [from, to] window in us."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = float(sys.argv[3]) if len(sys.argv) > 3 else 1e18
for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    if s < lo or s > hi:
        continue
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("pga::", "")
    print(f"q{r['Queue_Id']:>2} s{r['Stream_Id']:>2} {s:10.1f} {e:10.1f} {e - s:7.1f}  {n[:60]}")
