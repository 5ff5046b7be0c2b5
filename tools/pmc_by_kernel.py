"""Mean counter value per dispatch, per kernel name, over a rocprofv3 --pmc session directory:
    python3 tools/pmc_by_kernel.py gpurun_out/r06/g1"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            short = name.split("(")[0].replace("void ", "")
            grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
            acc[(f"{short} grid={grid}", r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{k:72s} {c:22s} n={len(v):3d} mean={sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
