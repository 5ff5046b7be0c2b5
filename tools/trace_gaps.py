"""Kernel durations and start-to-start intervals of one kernel name from a rocprofv3 kernel-trace
CSV: python tools/trace_gaps.py <kernel_trace.csv> <name substring>"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
s = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.int64)
e = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.int64)
o = np.argsort(s)
s, e = s[o][-400:], e[o][-400:]
d = (e - s) / 1e3
gap = (s[1:] - e[:-1]) / 1e3
iv = np.diff(s) / 1e3
print(f"{len(s)} launches: duration med {np.median(d):.2f} mean {d.mean():.2f} us | "
      f"gap med {np.median(gap):.2f} mean {gap.mean():.2f} us | interval mean {iv.mean():.2f} us")
