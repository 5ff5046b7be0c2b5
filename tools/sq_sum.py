"""Mean per-dispatch SQ counter values of the kernels matching a substring: python tools/sq_sum.py <dir> <substr>"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for x in csv.DictReader(open(f)):
        if sys.argv[2] in x["Kernel_Name"]:
            acc[x["Counter_Name"]].append(float(x["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
