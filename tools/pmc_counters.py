"""Per-kernel counter digest of a round-4 counter session (tools/r04_counters.sh) ->
<session>/counters.json, copied to profiles/counters.json for bench.py.

For every (workload, kernel) pair: the mean per-dispatch SQ counters of the two SQ passes, the
kernel's average duration from the same session's kernel trace, and derived
  mfma_busy_cycles_per_simd = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs (256 CUs x 4)
  busy_cycles_per_se        = SQ_BUSY_CYCLES / 32 shader engines (the kernel's span in shader cycles)
  mfma_busy_frac            = their ratio: the share of the kernel's span the matrix pipes are busy
  clock_ghz                 = busy_cycles_per_se / the kernel's average duration (profiled clock)
and, where a FETCH_SIZE / WRITE_SIZE pass exists, HBM bytes per launch corrected as
MI355X_MICROARCH.md prescribes for gfx950 (2 x FETCH_SIZE + WRITE_SIZE, KiB).  The first quarter
of the dispatches (cold caches, graph warm-up) is skipped.

    python3 tools/pmc_counters.py <session dir> <workload>:<kernel substring> ...
"""
import csv
import glob
import json
import os
import sys

SIMDS, SES = 1024, 32


def per_dispatch(root, kernel):
    vals = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r.get("Kernel_Name", ""):
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: v[len(v) // 4:] or v for k, v in vals.items()}


def mean(v):
    return sum(v) / len(v) if v else None


def kernel_avg_ns(session, workload, kernel):
    for f in glob.glob(os.path.join(session, f"trace_{workload}", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Name"]:
                return float(r["AverageNs"]), r["Name"], int(r["Calls"])
    return None, None, 0


def tree_src():
    """The source hash of the library the session ran (rk_build_info's src: the tree's csrc/ and
    include/ hash, rankops._lib.tree_source_hash), so bench.py can tell a stale counter entry."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd"))
    try:
        from rankops import _lib
        return _lib.tree_source_hash()
    except Exception:  # no torch here: leave the entry untagged
        return None


def main():
    session = sys.argv[1]
    out_path = os.path.join(session, "counters.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    src = tree_src()
    for spec in sys.argv[2:]:
        workload, kernel = spec.split(":", 1)
        e = {"session": os.path.basename(os.path.normpath(session)), "src": src}
        sq = {}
        for p in ("a", "b"):
            for k, v in per_dispatch(os.path.join(session, f"sq_{workload}", p), kernel).items():
                sq[k] = round(mean(v), 1)
        if sq:
            e["sq"] = sq
            mfma = sq.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / SIMDS
            span = sq.get("SQ_BUSY_CYCLES", 0) / SES
            e["mfma_busy_cycles_per_simd"] = round(mfma, 1)
            e["busy_cycles_per_se"] = round(span, 1)
            if span:
                e["mfma_busy_frac"] = round(mfma / span, 4)
        ns, name, calls = kernel_avg_ns(session, workload, kernel)
        if ns:
            e["trace_avg_ns"] = round(ns, 1)
            e["trace_kernel"] = name
            e["trace_calls"] = calls
            if e.get("busy_cycles_per_se"):
                e["clock_ghz"] = round(e["busy_cycles_per_se"] / ns, 3)
        fetch = per_dispatch(os.path.join(session, f"pmc_{workload}", "fetch"), kernel).get("FETCH_SIZE")
        write = per_dispatch(os.path.join(session, f"pmc_{workload}", "write"), kernel).get("WRITE_SIZE")
        if fetch and write:
            fk, wk = mean(fetch), mean(write)
            e["traffic"] = {"bytes_per_launch": round((2 * fk + wk) * 1024), "fetch_size_kib_raw": round(fk, 1),
                            "write_size_kib": round(wk, 1), "dispatches": [len(fetch), len(write)],
                            "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM)"}
        data[f"{workload}:{kernel}"] = e
        print(spec, json.dumps(e)[:400])
    json.dump(data, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
