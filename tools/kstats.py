#!/usr/bin/env python3
"""Short table of a rocprofv3 kernel_stats.csv: name, calls, avg/min/max us, share."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(f"== {path}")
    with open(path) as f:
        for r in csv.DictReader(f):
            n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", ""))
            n = re.sub(r"^.*::", "", n) if "<" not in n else re.sub(r"^[^<]*::(?=[^:<]*<)", "", n)
            print(f"{n[:48]:48s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:7.1f}us "
                  f"min={float(r['MinNs'])/1e3:7.1f} max={float(r['MaxNs'])/1e3:7.1f} {float(r['Percentage']):5.1f}%")
