"""Summarise rocprofv3 kernel traces: per-kernel average duration over the last `--last`
dispatches of each kernel (graph replays), grouped per trace file."""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--last", type=int, default=40)
    args = ap.parse_args()
    files = []
    for p in args.paths:
        files += sorted(glob.glob(os.path.join(p, "*kernel_trace.csv"))) if os.path.isdir(p) else [p]
    for f in files:
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        by = collections.OrderedDict()
        for r in rows:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            by.setdefault(r["Kernel_Name"], []).append(d)
        print(f"== {f}")
        tot = 0.0
        for k, ds in by.items():
            ds = ds[-args.last:]
            avg = sum(ds) / len(ds)
            if "rk::" not in k and avg < 1.0:
                continue
            tot += avg
            print(f"  {avg:9.2f} us  x{len(by[k]):4d}  {k[:110]}")
        print(f"  {tot:9.2f} us  total of listed kernel averages")


if __name__ == "__main__":
    main()
