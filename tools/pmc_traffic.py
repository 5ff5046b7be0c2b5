"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes -> profiles/traffic.json.

Run on the GPU box (two separate --pmc passes, kernel trace only, as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes):

    rocprofv3 --pmc FETCH_SIZE -d OUT/fetch -o run --output-format csv -- python3 tools/kprof.py --workload din
    rocprofv3 --pmc WRITE_SIZE -d OUT/write -o run --output-format csv -- python3 tools/kprof.py --workload din
    python3 tools/pmc_traffic.py OUT din din_forward_kernel

gfx950 correction (same section): FETCH_SIZE counts 64 B per 128-B request of a wide
coalesced read, i.e. half the bytes, so it is doubled; WRITE_SIZE is taken as is.  Both are
in KiB.  The raw values are kept next to the corrected total.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(root, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and kernel in r.get("Kernel_Name", ""):
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    out_dir, workload, kernel = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = per_dispatch(os.path.join(out_dir, "fetch"), "FETCH_SIZE", kernel)
    write = per_dispatch(os.path.join(out_dir, "write"), "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit(f"no {kernel} dispatches with counters under {out_dir}")
    # skip the first dispatches (cold caches / graph warm-up), average the rest
    f = fetch[len(fetch) // 4:] or fetch
    w = write[len(write) // 4:] or write
    fetch_kib, write_kib = sum(f) / len(f), sum(w) / len(w)
    total = (2 * fetch_kib + write_kib) * 1024
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    data = {}
    if os.path.exists(path):
        data = json.load(open(path))
    data[f"{workload}:{kernel}"] = {"bytes_per_launch": round(total), "fetch_size_kib_raw": round(fetch_kib, 1),
                                    "write_size_kib": round(write_kib, 1), "dispatches": [len(fetch), len(write)],
                                    "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM)"}
    json.dump(data, open(path, "w"), indent=1)
    print(json.dumps(data[f"{workload}:{kernel}"]))


if __name__ == "__main__":
    main()
