"""Top kernels of a rocprofv3 *_kernel_stats.csv: name, calls, average us, share of total time."""
import csv
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"== {f}: {tot / 1e3:.1f} us total")
    for r in rows[:25]:
        print(f"{r['Name'][:84]:84s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:9.1f} "
              f"{100 * float(r['TotalDurationNs']) / tot:5.1f}")
