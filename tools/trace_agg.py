"""Per-(kernel, grid) aggregate of a rocprofv3 kernel trace: calls, average and total µs.
Usage: python tools/trace_agg.py <kernel_trace.csv> [steps] [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
agg = collections.defaultdict(list)
for x in rows:
    k = (x["Kernel_Name"][:64], x["Grid_Size_X"], x["Grid_Size_Y"], x["Grid_Size_Z"])
    agg[k].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{k[0]:64s} g=({k[1]},{k[2]},{k[3]}) n={len(v):4d} avg={sum(v) / len(v):7.1f} per-step={sum(v) / steps:7.1f}")
print(f"total per step {tot / steps:.1f} us")
