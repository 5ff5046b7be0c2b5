"""rankops benchmark — forward samples/s of the CTR interaction engine on MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, one process per GPU
(torchrun for N > 1); rank 0 prints ONE JSON line.

Workload (BASELINE.json metric "forward samples/sec at batch 4096 (DCN, DIN, BST)"): the
headline is configs[2], DIN forward with behaviour seq_len 50, emb_dim 32, batch 4096 per GPU,
wechat-sized tables, eval mode, inputs resident in HBM.  A step is one forward of one batch,
captured once in a hipGraph and replayed.  The H2 attention MLP is in 'frozen' mode (drawn once
with the reference's calls, kept on the device); the per-call redraw is reported separately
under models.din_per_call (eager, it has host work).  Multi-GPU is replicas (the forward has
no exchange step): every rank runs its own batch, `value` = all ranks' samples / max time.

Extra keys: `models` (N=1, rank 0) times DCN@4096, DeepFM configs[1] and BST configs[3] the
same way; `roofline` prices the dominant kernel with HIP events around its own launches on the
stream it runs on; `cpu_baseline` times the oracle (CPU restatement, per-call draws included)
on a bounded sample of the same workload on this host; `loader` times the host input path
(raw ID strings -> bucketed batch on the GPU -> forward, rankops.loader) against the reference's
per-row Python Dataset logic; `eval_metrics` times evaluate()'s loss / accuracy / AUC over 256
eval batches on the device (rankops.EvalAccumulator) against the reference's host-copy + sklearn path.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd")
for _p in (PKG_DIR, REPO, os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_FP32_MFMA = 157.3e12  # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_HBM = 8.0e12          # MI355X_MICROARCH.md: HBM3E peak BW (spec)

METRIC = "forward samples/sec at batch 4096 (DCN, DIN, BST) on 1/2/4/8 MI355X"

# Algorithmic work per sample
DIN_ATT_FLOP = 2 * 50 * (128 * 64 + 64 * 32 + 32)  # 1,027,200: att-MLP of din_attention, T=50, H=32
DIN_FWD_FLOP = DIN_ATT_FLOP + 6_400 + 444_672       # whole DIN forward, reference formulation
# what din_forward_kernel<32> issues per sample: split layer 1 (K=H) + layer 2 + layer 3 over 64 padded
# positions, the per-sample bias u, and the fcn at padded widths (128->512->256->128)
DIN_FWD_EXEC_FLOP = 2 * 64 * (32 * 64 + 64 * 32 + 32) + 2 * 64 * 32 + 2 * (128 * 512 + 512 * 256 + 256 * 128)
DEEPFM_GATHER_BYTES = 30 * (8 + 128 + 4) + 30 * 128 + 8  # 8,048 B: gather+FM kernel
BST_BLOCK_FLOP = 14_680_064
FWFM_BYTES_PER_SAMPLE = 6 * (8 + 32 + 4) + 4
DCN_FLOP = 379_236
ZIPF_A = 1.1  # Zipf(1.1) index variant for cache sensitivity


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--din-streams", type=int, default=1,
                    help="DIN headline: batches in flight on as many HIP streams (default 1; "
                         "tools/din_streams.py measures 2-4)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--no-extras", action="store_true", help="skip the per-model extras")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-sharded", action="store_true", help="skip the table-sharded DeepFM (configs[4])")
    ap.add_argument("--no-model-curve", action="store_true", help="skip the modelled 1->8 GPU curve of configs[4]")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--models", default="dcn,dcn_per_call,dcn_256_per_call,deepfm,bst,bst_ref,fwfm,afm,deepcrossing,"
                                        "din_per_call,din_zipf,dcn_eager,din_eager,deepfm_eager,bst_eager")
    ap.add_argument("--no-loader", action="store_true", help="skip the host input-path (bucketing) leg")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step legs")
    ap.add_argument("--details", default=DEFAULT_DETAILS,
                    help="file for the full result (every leg); the stdout line is the compact summary")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # one GPU per rank; modulo the visible devices only so that a one-GPU box can rehearse the
        # N > 1 path with every rank on its single GPU (timings then meaningless)
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        # a bounded collective timeout: a rank that fails between collectives ends the job within
        # minutes instead of leaving the others blocked until the driver's limit
        timeout = datetime.timedelta(seconds=int(os.environ.get("RANKOPS_BENCH_PG_TIMEOUT", "300")))
        if os.environ.get("RANKOPS_BENCH_BACKEND") == "gloo":
            # rehearsal only (RCCL refuses two ranks on one GPU): gloo with the tensors on the GPU
            dist.init_process_group("gloo", timeout=timeout)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(world, value: float) -> float:
    if world == 1:
        return value
    import torch.distributed as dist
    t = torch.tensor([value], device="cuda", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ------------------------------------------------------------------ workloads

def workload(name: str, batch: int, seed: int, zipf: float = None):
    """(model, inputs, call, cfg) for a benchmark workload, built directly on the GPU.  `zipf`:
    table indices drawn from Zipf(zipf) popularity instead of uniformly."""
    import helpers as H
    dev = torch.device("cuda", torch.cuda.current_device())
    name = name[:-len("_eager")] if name.endswith("_eager") else name
    if name in ("din", "din_per_call"):
        cfg = {"vocab": H.WECHAT_VOCAB, "T": 50, "dim": 32,
               "interaction_weights": "frozen" if name == "din" else "per_call"}
        model_name = "din"
    elif name in ("dcn", "dcn_per_call", "dcn_256_per_call"):
        cfg = {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen" if name == "dcn" else "per_call"}
        model_name = "dcn"
    elif name == "deepfm":
        cfg = {"dim": 32, "fields": {f"field_{i:02d}": 1_000_000 for i in range(30)}}
        model_name = "deepfm"
    elif name == "bst":
        cfg = {"vocab": H.WECHAT_VOCAB, "T": 64, "dim": 128, "heads": 4, "max_len": 64}
        model_name = "bst"
    elif name == "bst_ref":  # the reference script's own shape: d_model 16 (bst.py:192,339-349), 4 heads, T 50
        cfg = {"vocab": H.WECHAT_VOCAB, "T": 50, "dim": 16, "heads": 4, "max_len": 50}
        model_name = "bst"
    elif name == "fwfm":
        cfg = {"vocab": H.WECHAT_VOCAB, "dim": 8}
        model_name = "fwfm"
    elif name == "afm":  # afm.py:241-242 defaults: embedding_dim 8, attention_factor 128
        cfg = {"vocab": H.WECHAT_VOCAB, "dim": 8, "att": 128}
        model_name = "afm"
    elif name == "deepcrossing":  # deepcrossing.py:319-320 defaults: residual_internal_dim 128, 1 unit
        cfg = {"vocab": H.WECHAT_VOCAB, "internal": 128, "units": 1, "interaction_weights": "frozen"}
        model_name = "deepcrossing"
    else:
        raise ValueError(name)
    with torch.device(dev):
        model = H.build(model_name, cfg, seed=42)
    model = model.to(dev).eval()
    if zipf is not None:
        cfg = dict(cfg, zipf=zipf)
    inp = H.to_device(H.make_inputs(model_name, cfg, batch, seed=1000 + seed), dev)
    return model, inp, (lambda: H.call_model(model, model_name, inp)), cfg, model_name


def graph_of(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    # thread_local: with a process group up, RCCL's watchdog thread keeps querying its events
    # during a capture; only this thread's calls are restricted
    with torch.no_grad(), torch.cuda.graph(g, capture_error_mode="thread_local"):
        out = fn()
    return g, out


def time_replays(run, steps, warmup, world):
    for _ in range(warmup):
        run()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def kernel_avg_ms(launch, iters=50):
    """Average duration of one launch, HIP events on the stream the kernel runs on."""
    st = torch.cuda.current_stream()
    for _ in range(5):
        launch()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record(st)
    for _ in range(iters):
        launch()
    end.record(st)
    end.synchronize()
    return start.elapsed_time(end) / iters


def graph_kernel_avg_ms(launch, per_graph=20, iters=10):
    """Average device time of one launch of a short kernel: `per_graph` back-to-back launches
    captured in one hipGraph, replayed `iters` times, HIP events on the replay stream (host
    launch cost excluded; the ~1.5 us dependent-kernel boundary per launch included)."""
    g, _ = graph_of(lambda: [launch() for _ in range(per_graph)])
    st = torch.cuda.current_stream()
    g.replay()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record(st)
    for _ in range(iters):
        g.replay()
    end.record(st)
    end.synchronize()
    return start.elapsed_time(end) / (iters * per_graph)


# ------------------------------------------------------------------ PMC traffic (profiles/traffic.json)

COUNTERS_FILE = os.path.join("profiles", "counters.json")  # tools/r04_counters.sh -> tools/pmc_counters.py


_LIB_SRC = None  # the loaded librankops.so's source hash (rk_build_info), set in main()


def counter_staleness(e: dict) -> str:
    """Whether a committed counter entry was collected on the library now loaded: "current" when
    the entry's `src` (the tree source hash at collection, tools/pmc_counters.py) equals the
    loaded library's, "stale (<src>)" when it differs, "unknown" for entries that predate the tag."""
    src = e.get("src")
    if not src or not _LIB_SRC:
        return "unknown"
    return "current" if src == _LIB_SRC else f"stale ({src})"


def load_counters(kernel: str, workload_name: str):
    """The committed counter digest of `kernel` under `workload_name` (profiles/counters.json: SQ
    MFMA-busy and wait counters, the profiled average duration, PMC HBM bytes), or None."""
    try:
        with open(os.path.join(REPO, COUNTERS_FILE)) as f:
            e = json.load(f).get(f"{workload_name}:{kernel}")
    except (OSError, ValueError):
        return None
    if e is not None:
        e = dict(e, file=COUNTERS_FILE, staleness=counter_staleness(e))
    return e


def load_traffic(kernel: str, workload_name: str):
    """PMC-measured HBM bytes per launch of `kernel` (profiles/counters.json)."""
    e = load_counters(kernel, workload_name)
    if not e or "traffic" not in e:
        return None
    return dict(e["traffic"], file=COUNTERS_FILE, session=e["traffic"].get("session", e.get("session")),
                staleness=e["staleness"])


def counter_fields(kernel: str, workload_name: str, flop_per_launch: float = None):
    """mfma_busy_frac and the profiled duration (plus the roofline fraction at that duration)
    from the committed counter digest, for a bench roofline block."""
    e = load_counters(kernel, workload_name)
    if not e:
        return {"mfma_busy_frac": None, "counters": None}
    out = {"mfma_busy_frac": e.get("mfma_busy_frac"),
           "counters": {k: e.get(k) for k in ("file", "session", "staleness", "mfma_busy_cycles_per_simd",
                                              "busy_cycles_per_se", "clock_ghz", "trace_avg_ns")}}
    if flop_per_launch and e.get("trace_avg_ns"):
        out["frac_at_profiled_duration"] = round(flop_per_launch / (e["trace_avg_ns"] * 1e-9) / PEAK_FP32_MFMA, 4)
    return out


# ------------------------------------------------------------------ CPU baseline (oracle)

def _frozen_interaction(name, cfg):
    """H2 weights drawn once in oracle form (the CPU counterpart of interaction_weights='frozen')."""
    from oracle import reference_forward as ref
    if name == "din":
        return ref.draw_din_att(cfg.get("dim", 16))
    if name == "dcn":
        return ref.draw_cross(16 + 16 + 2 + 4 * 4, cfg.get("cross", 1))
    return None


def cpu_baseline(name, model, cfg, batch, budget_s, frozen, threads=None):
    """The oracle (CPU restatement of the reference forward) on this host, on a bounded sample:
    repeated forwards of batch `batch` until ~budget_s.  `frozen` times the same H2 mode as the
    GPU headline (interaction MLP drawn once); otherwise every call redraws it from the CPU
    generator as the reference does."""
    import helpers as H
    n = threads or min(16, len(os.sched_getaffinity(0)))
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(n)
    p = H.cpu_params(model)
    cfg_cpu = dict(cfg)
    inp = H.make_inputs(name, cfg_cpu, batch, seed=2000)
    inter = _frozen_interaction(name, cfg_cpu) if frozen else None
    with torch.no_grad():
        H.call_oracle(name, cfg_cpu, p, inp, inter)  # warm-up
        t0 = time.perf_counter()
        iters = 0
        while True:
            H.call_oracle(name, cfg_cpu, p, inp, inter)
            iters += 1
            el = time.perf_counter() - t0
            if el >= budget_s or iters >= 2000:
                break
    torch.set_num_threads(prev_threads)
    mode = "H2 weights frozen (drawn once)" if frozen else "per-call H2 draws included"
    return {"value": round(iters * batch / el, 1), "unit": "samples/s", "cores": n, "kind": "port",
            "sample": f"{iters} oracle {name.upper()} forwards of batch {batch} ({el:.1f} s, {mode}, fp32, "
                      f"eval + no_grad, torch {torch.__version__} CPU)"}


def cpu_baselines(model, cfg, head_value, extras, batch, budget_s):
    """cpu_baseline for the headline (DIN configs[2], same frozen H2 mode as the GPU line), plus
    the per-call mode beside din_per_call, DCN at batch 4096 (the north star's >= 10x target) in
    both modes beside models.dcn / models.dcn_per_call, and configs[0] (DCN, wechat schema,
    batch 256, the reference's CPU plumbing with per-call draws)."""
    import helpers as H
    out = cpu_baseline("din", model, cfg, batch, budget_s, frozen=True)
    out["gpu_over_cpu"] = round(head_value / out["value"], 1)
    out["mode"] = "frozen H2 beside the frozen GPU headline"
    legs = {}
    leg = cpu_baseline("din", model, cfg, batch, budget_s / 3, frozen=False)
    if "din_per_call" in extras:
        leg["gpu_samples_per_s"] = extras["din_per_call"]["samples_per_s"]
        leg["gpu_over_cpu"] = round(leg["gpu_samples_per_s"] / leg["value"], 1)
    legs["din_per_call"] = leg
    dcn_cfg = {"vocab": H.WECHAT_VOCAB}
    dcn = H.build("dcn", dcn_cfg, seed=42)
    for key, b, frozen, gpu_key in (("dcn_4096", 4096, True, "dcn"), ("dcn_4096_per_call", 4096, False,
                                                                       "dcn_per_call"),
                                    ("configs0_dcn_256", 256, False, "dcn_256_per_call")):
        leg = cpu_baseline("dcn", dcn, dcn_cfg, b, budget_s / (1.5 if key == "dcn_4096" else 3), frozen)
        if gpu_key in extras:
            leg["gpu_samples_per_s"] = extras[gpu_key]["samples_per_s"]
            leg["gpu_over_cpu"] = round(leg["gpu_samples_per_s"] / leg["value"], 1)
        legs[key] = leg
    legs["dcn_4096"]["target"] = ">= 10x (BASELINE.json north star, DCN batch 4096, 1 MI355X)"
    # single-threaded ("It is also reported single-threaded")
    for key, nm, mdl, c, b, gpu_v in (("din_1thread", "din", model, cfg, batch, head_value),
                                      ("dcn_4096_1thread", "dcn", dcn, dcn_cfg, 4096,
                                       extras.get("dcn", {}).get("samples_per_s"))):
        leg = cpu_baseline(nm, mdl, c, b, budget_s / 3, True, threads=1)
        if gpu_v:
            leg["gpu_samples_per_s"] = gpu_v
            leg["gpu_over_cpu"] = round(gpu_v / leg["value"], 1)
        legs[key] = leg
    out["legs"] = legs
    return out


# ------------------------------------------------------------------ configs[4]: table-sharded DeepFM

SHARDED_FIELDS = 30
SHARDED_ROWS_PER_FIELD = 3_333_334  # 30 x 3,333,334 = 1.0e8 rows (second- and first-order tables)
SHARDED_GLOBAL_BATCH = 65536


def bench_sharded(world, rank, steps, warmup):
    """Strong scaling: global batch 65536 split over the ranks, 1e8 embedding rows split by field.
    At world > 1 the local batch runs as ShardedDeepFM's exchange pipeline (pipeline_chunks
    chunks; per chunk three captured hipGraph segments with asynchronous RCCL all-to-alls between
    them); at world 1 the forward is one hipGraph (nothing to exchange)."""
    import helpers as H
    from rankops.sharded import ShardedDeepFM, row_stride
    dev = torch.device("cuda", torch.cuda.current_device())
    fields = {f"field_{i:02d}": SHARDED_ROWS_PER_FIELD for i in range(SHARDED_FIELDS)}
    torch.manual_seed(42)
    with torch.device(dev):
        model = ShardedDeepFM(fields, 32, [512, 256, 128], rank=rank, world_size=world)
    H.randomize_eval_stats(model, 43)
    model.eval()
    B_l = SHARDED_GLOBAL_BATCH // world
    rng = np.random.default_rng(5000 + rank)
    cat = {f: torch.from_numpy(rng.integers(0, SHARDED_ROWS_PER_FIELD, B_l, dtype=np.int64)).to(dev) for f in fields}
    if world == 1:  # nothing to exchange: one packed FM gather + the tail, one hipGraph
        g0, _ = graph_of(lambda: model.run_steps(cat))
        step = g0.replay
    else:
        # the cross-batch exchange pipeline (ShardedDeepFM.pipeline, captured): per step the index
        # all-to-all of batch i, the gather + row all-to-all of batch i-1 (RCCL async) and the
        # one-launch forward of batch i-2; three local batches bound to
        # the pipeline's slots.  Warm-up fills the pipeline; every timed step completes one batch.
        cats = [cat] + [{f: torch.from_numpy(rng.integers(0, SHARDED_ROWS_PER_FIELD, B_l, dtype=np.int64)).to(dev)
                         for f in fields} for _ in range(2)]
        # side_stream=False: pack and gather in stream order before the forward (a gather beside the
        # forward displaces its one-per-CU workgroups: sharded_model_curve's step_two_streams)
        step = model.pipeline(B_l, capture=cats, side_stream=False).step

    t = max_over_ranks(world, time_replays(step, steps, max(warmup, 3), world))
    # bytes this rank sends per step (indices + rows: row_splits' input splits), (P-1)/P of them to peers
    wire = (B_l * SHARDED_FIELDS * model.index_dtype.itemsize + sum(model.row_splits(B_l)[1]) * 4) * (world - 1) / world
    return {"samples_per_s": round(SHARDED_GLOBAL_BATCH * steps / t, 1), "ms_per_step": round(1e3 * t / steps, 4),
            "global_batch": SHARDED_GLOBAL_BATCH, "rows_total": SHARDED_FIELDS * SHARDED_ROWS_PER_FIELD,
            "fields_per_rank": len(model.local_fields), "wire_bytes_per_rank_step": int(wire),
            "wire_format": "split" if model.split_wire() else "packed",
            "scaling": "strong",
            "mode": ("one hipGraph (packed FM gather + tail, no exchange at P=1)" if world == 1 else
                     "cross-batch pipeline (ShardedDeepFM.pipeline, side_stream=False): per step pack + index "
                     "all_to_all_single of batch i, gather + row all_to_all_single of batch i-1, the one-launch "
                     "forward of batch i-2, local steps in stream order as hipGraphs, the all-to-alls async on "
                     "RCCL's stream between them")}


XGMI_LINK_BPS = 153e9   # MI355X: 7 xGMI links x ~153 GB/s per GPU, point to point (fully connected node)
A2A_LATENCY_S = 20e-6   # assumed fixed cost per RCCL all_to_all_single call (not measured here)


def sharded_model_curve(p1_ms: float, ps=(2, 4, 8), chunks=4, iters=20):
    """A MODEL, not a measurement, of the 1 -> 8 GPU strong-scaling curve of configs[4] (global
    batch 65536, 1e8 rows), built from what one GPU can time: rank 0's local device work at P
    ranks, captured as hipGraphs and timed here, plus the wire time of the two all-to-alls from
    their per-link bytes at XGMI_LINK_BPS (each peer pair has its own link) and an assumed
    A2A_LATENCY_S per collective.  Three columns:
      serial      the chunked run_steps (pack, per chunk: gather + row exchange + forward), all summed;
      overlapped  the same with chunk c's row exchange hidden behind chunk c+1's gather and chunk
                  c-1's forward (round 4's design);
      pipelined   ShardedDeepFM.pipeline (round 5): the index and row exchanges of batches i and
                  i-1 run under batch i-2's forward, so a step costs max(local device work, wire +
                  per-call latency); the local device work is pack + ONE gather over all P x B_l
                  rows + ONE forward launch over B_l, timed back to back as one hipGraph, plus the
                  measured slowdown of the forward while a side-stream copy of the row exchange's
                  bytes runs beside it (a stand-in for RCCL's copy kernels taking CUs)."""
    import helpers as H
    from rankops.sharded import ShardedDeepFM, row_stride
    dev = torch.device("cuda", torch.cuda.current_device())
    fields = {f"field_{i:02d}": SHARDED_ROWS_PER_FIELD for i in range(SHARDED_FIELDS)}
    RS = row_stride(32)
    curve = {"1": {"ms_per_step": p1_ms, "samples_per_s": round(SHARDED_GLOBAL_BATCH / (p1_ms * 1e-3), 1),
                   "kind": "measured (sharded_deepfm at P = 1)"}}
    for P in ps:
        torch.manual_seed(42)
        with torch.device(dev):
            model = ShardedDeepFM(fields, 32, [512, 256, 128], rank=0, world_size=P)
        H.randomize_eval_stats(model, 43)
        model.eval()
        B_l = SHARDED_GLOBAL_BATCH // P
        C = len(model.chunk_bounds(B_l, chunks))
        B_c = B_l // C
        F_me = len(model.local_fields)
        rng = np.random.default_rng(77 + P)
        recv_idx = torch.from_numpy(rng.integers(0, SHARDED_ROWS_PER_FIELD, P * B_l * F_me)).to(
            dev, model.index_dtype)
        recv_rows = torch.randn(sum(model.row_splits(B_c)[0]), device=dev)
        recv_full = torch.randn(sum(model.row_splits(B_l)[0]), device=dev)
        cat = {f: torch.from_numpy(rng.integers(0, SHARDED_ROWS_PER_FIELD, B_l)).to(dev) for f in fields}
        with torch.no_grad():
            g_pack, _ = graph_of(lambda: model.pack_indices(cat))
            g_gather, _ = graph_of(lambda: model.gather_rows(recv_idx, B_l, 0, B_c))
            g_fm, _ = graph_of(lambda: model.fm_and_tail(recv_rows, B_c))
            g_gather1, rows1 = graph_of(lambda: model.gather_rows(recv_idx, B_l, 0, B_l))
            g_fm1, _ = graph_of(lambda: model.fm_and_tail(recv_full, B_l))
            g_seq, _ = graph_of(lambda: (model.pack_indices(cat), model.gather_rows(recv_idx, B_l, 0, B_l),
                                         model.fm_and_tail(recv_full, B_l)))
        t_pack = kernel_avg_ms(g_pack.replay, iters)
        t_gather = kernel_avg_ms(g_gather.replay, iters) * C
        t_fm = kernel_avg_ms(g_fm.replay, iters) * C
        t_gather1 = kernel_avg_ms(g_gather1.replay, iters)
        t_fm1 = kernel_avg_ms(g_fm1.replay, iters)
        t_seq = kernel_avg_ms(g_seq.replay, iters)
        # contention proxy: the forward with a copy of the bytes this rank's RCCL kernels move
        # (P2P writes: (P-1)/P of its send rows out to the peers; the peers' kernels push its
        # receive rows) on a second stream, which takes CUs from the forward as RCCL's would
        xfer = int(sum(model.row_splits(B_l)[1]) * (P - 1) / P)
        src, dst = torch.empty(xfer, device=dev), torch.empty(xfer, device=dev)
        side = torch.cuda.Stream()

        def fwd_with_copy():
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                dst.copy_(src)
            g_fm1.replay()
            torch.cuda.current_stream().wait_stream(side)
        t_fm1_copy = kernel_avg_ms(fwd_with_copy, iters)
        contention = max(0.0, t_fm1_copy - t_fm1)

        # one steady-state step of the cross-batch pipeline on one GPU: the forward of batch i-2 on
        # the compute stream while the side stream packs batch i, gathers batch i-1 and then moves
        # that rank's row-exchange bytes (the stand-in for RCCL's copy kernels); the side work takes
        # CUs as the forward's workgroups retire
        def step_stand_in():
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                g_pack.replay()
                g_gather1.replay()
                dst.copy_(src)
            g_fm1.replay()
            torch.cuda.current_stream().wait_stream(side)
        t_step = kernel_avg_ms(step_stand_in, iters)
        t_comp = t_pack + t_gather + t_fm
        # per link: this rank's bytes to one peer (F / P fields of its B_l samples, each way)
        f_peer = SHARDED_FIELDS / P
        idx_link = B_l * f_peer * model.index_dtype.itemsize
        rows_link = sum(model.row_splits(B_l)[0]) * 4 / P  # one owner's block per peer link
        t_idx = 1e3 * (idx_link / XGMI_LINK_BPS + A2A_LATENCY_S)  # one index exchange per step
        t_rows = 1e3 * (rows_link / XGMI_LINK_BPS + C * A2A_LATENCY_S)
        serial = t_comp + t_idx + t_rows
        # chunked pipeline: pack + index exchange, then chunk c's rows travel behind chunk c+1's gather and
        # chunk c-1's FM + tail; the first chunk's gather and the last chunk's exchange stay exposed
        overlap = t_pack + t_idx + max(t_gather + t_fm, t_rows) + (t_gather + t_rows) / C
        # cross-batch pipeline: one row exchange per step (one call), hidden behind the forward
        wire1 = 1e3 * ((idx_link + rows_link) / XGMI_LINK_BPS + 2 * A2A_LATENCY_S)
        # the pipeline's schedule (ShardedDeepFM.pipeline(side_stream=False), the bench's): pack and
        # gather in stream order before the forward, only the collectives beside it -> the serial local
        # work plus the forward's measured slowdown under the exchange's copy traffic; gather and
        # forward on two streams (step_two_streams) measured slower: the gather's workgroups displace
        # the forward's one-per-CU workgroups
        local1 = min(t_seq + contention, t_step)
        piped = max(local1, wire1)
        piped_free = max(t_seq, wire1)  # serial local work, RCCL's kernels on idle CUs (no contention)
        curve[str(P)] = {
            "kind": "model, not a measurement",
            "B_local": B_l, "fields_rank0": F_me, "chunks": C,
            "compute_ms": {"pack": round(t_pack, 4), "gather_local": round(t_gather, 4),
                           "fm_and_tail": round(t_fm, 4)},
            "pipelined_compute_ms": {"pack": round(t_pack, 4), "gather_one_launch": round(t_gather1, 4),
                                     "forward_one_launch": round(t_fm1, 4),
                                     "pack_gather_forward_one_graph": round(t_seq, 4),
                                     "forward_with_copy_beside": round(t_fm1_copy, 4),
                                     "contention": round(contention, 4), "copy_bytes": 4 * xfer,
                                     "step_two_streams": round(t_step, 4)},
            "wire_ms": {"index": round(t_idx, 4), "rows": round(t_rows, 4), "pipelined_per_step": round(wire1, 4)},
            "bytes_per_link": {"index": int(idx_link), "rows": int(rows_link)},
            "wire_format": "split" if model.split_wire() else "packed",
            "ms_per_step": {"serial": round(serial, 4), "overlapped": round(overlap, 4), "pipelined": round(piped, 4),
                            "pipelined_no_contention": round(piped_free, 4)},
            "samples_per_s": {"serial": round(SHARDED_GLOBAL_BATCH / (serial * 1e-3), 1),
                              "overlapped": round(SHARDED_GLOBAL_BATCH / (overlap * 1e-3), 1),
                              "pipelined": round(SHARDED_GLOBAL_BATCH / (piped * 1e-3), 1)},
            "speedup_vs_p1": {"serial": round(p1_ms / serial, 2), "overlapped": round(p1_ms / overlap, 2),
                              "pipelined": round(p1_ms / piped, 2),
                              "pipelined_no_contention": round(p1_ms / piped_free, 2)},
            "pipelined_bound": "device" if local1 >= wire1 else "wire",
        }
        del model, g_pack, g_gather, g_fm, g_gather1, g_fm1, g_seq, rows1, src, dst, step_stand_in, fwd_with_copy
        torch.cuda.empty_cache()
    return {"assumptions": f"up to {chunks} chunks of >= 4096 samples (serial / overlapped); pipelined: one gather "
                           f"and one forward launch per step, exchanges of the two younger batches under the "
                           f"oldest one's forward; {XGMI_LINK_BPS / 1e9:.0f} GB/s per xGMI link, one link per "
                           f"peer pair; {A2A_LATENCY_S * 1e6:.0f} us per all_to_all_single call (assumed); "
                           "rank 0 (the most fields) timed; kernels of the other ranks equal or shorter; pipelined "
                           "= max(wire + 2 calls, one measured steady-state step: the forward on the compute "
                           "stream while a second stream packs, gathers and copies the rank's row-exchange "
                           "bytes, a stand-in for RCCL's copy kernels taking CUs)",
            "curve": curve}


# ------------------------------------------------------------------ host input path

def bench_loader(model, batch, batches=8):
    """Raw wechat rows -> DIN forward: C++ bucketing of Arrow string columns into one pinned
    buffer + one H2D copy (rankops.BatchAssembler), then the forward; against the reference's
    per-row Python Dataset + collate logic (oracle/bucketing.py, no pandas iloc) on this host.
    Synthetic vocabularies at the wechat row counts, ids in the `<field>_<id>` format, histories
    of U[1, 50] items."""
    import tempfile
    import pyarrow as pa
    import helpers as H
    import rankops
    from oracle import bucketing as ob
    rng = np.random.default_rng(77)
    tmp = tempfile.mkdtemp(prefix="rk_vocab_")
    words = {}
    for f, n in H.WECHAT_VOCAB.items():
        words[f] = [f"{f}_{i}" for i in rng.permutation(2 * n)[:n]]
        with open(os.path.join(tmp, ob.VOCAB_FILES[f]), "w") as fh:
            fh.write("".join(w + "\n" for w in words[f]))
    tables = []
    for b in range(batches):
        cols = {}
        for f, w in words.items():
            cols[f] = pa.array([w[i] for i in rng.integers(0, len(w), batch)], type=pa.string())
        feed = words["feedid"]
        cols[ob.DIN_SEQ] = pa.array([",".join(feed[j] for j in rng.integers(0, len(feed), int(n)))
                                     for n in rng.integers(1, 51, batch)], type=pa.string())
        for f in ob.DENSE_FEATURES:
            cols[f] = pa.array(np.log1p(rng.poisson(2.0, batch)).astype(np.float64))
        tables.append(pa.table(cols))
    vocabs = rankops.wechat_vocabularies(tmp)
    threads = min(16, len(os.sched_getaffinity(0)))
    res = {}
    for mode in ("device", "host"):
        asm = rankops.BatchAssembler("din", vocabs, device="cuda", bucketing=mode)
        for t in tables[:2]:
            asm(t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in tables:
            asm(t)
        torch.cuda.synchronize()
        t_asm = time.perf_counter() - t0
        with torch.no_grad():
            for t in tables[:2]:
                model(*asm(t))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in tables:
                model(*asm(t))
            torch.cuda.synchronize()
        t_e2e = time.perf_counter() - t0
        res[mode] = {"assemble_rows_per_s": round(batches * batch / t_asm, 1),
                     "end_to_end_samples_per_s": round(batches * batch / t_e2e, 1)}
    # the reference's Dataset + din_collate_fn logic, per row in Python, on one batch
    ovocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(tmp, ob.VOCAB_FILES[f]))) for f in ob.VOCAB_FILES}
    rows = tables[0].to_pylist()
    t0 = time.perf_counter()
    ob.batch("din", rows, ovocabs)
    t_py = time.perf_counter() - t0
    return {"device_bucketing": res["device"], "host_bucketing": res["host"],
            "python_dataset_rows_per_s": round(batch / t_py, 1), "batch": batch, "host_threads": threads,
            "avg_history_items": 25.5,
            "path": "Arrow string columns -> (device: raw bytes in one pinned buffer -> one H2D copy -> "
                    "rk_bucketize*_device | host: rk_bucketize* into the pinned buffer -> one H2D copy) -> "
                    "DIN forward (eager, frozen H2)"}


def bench_metrics(batch, batches=256):
    """evaluate()'s metric bookkeeping over `batches` eval batches already on the GPU: rankops
    EvalAccumulator (rk_eval_batch per batch, rk_auc once) against the reference's path
    (dcn.py:227-237: loss.item() + .cpu().numpy() per batch, then sklearn accuracy / roc_auc)."""
    import rankops
    from sklearn.metrics import accuracy_score, roc_auc_score
    g = torch.Generator(device="cuda").manual_seed(5)
    logits = [torch.randn(batch, device="cuda", generator=g) * 2 for _ in range(batches)]
    probs = [torch.sigmoid(x) for x in logits]
    labels = [(torch.rand(batch, device="cuda", generator=g) < 0.3).float() for _ in range(batches)]
    n = batch * batches

    def device_eval():
        acc = rankops.EvalAccumulator.for_model("dcn", "cuda")
        for p, y, x in zip(probs, labels, logits):
            acc.add(p, y, logits=x)
        return acc.result()

    device_eval()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = device_eval()
    t_dev = time.perf_counter() - t0
    # the AUC kernel chain alone, on the concatenated scores
    cat_p, cat_y = torch.cat(probs), torch.cat(labels)
    rankops.roc_auc(cat_p, cat_y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        rankops.roc_auc(cat_p, cat_y)
    torch.cuda.synchronize()
    t_auc = (time.perf_counter() - t0) / 10

    crit = torch.nn.BCEWithLogitsLoss()
    t0 = time.perf_counter()
    total, all_l, all_p = 0.0, [], []
    for p, y, x in zip(probs, labels, logits):
        total += crit(x, y).item()
        all_l.extend(y.cpu().numpy())
        all_p.extend(p.cpu().numpy())
    ref = (total / batches, accuracy_score(all_l, np.round(all_p)), roc_auc_score(all_l, all_p))
    t_ref = time.perf_counter() - t0
    return {"rows": n, "batches": batches, "device_eval_ms": round(1e3 * t_dev, 2),
            "device_rows_per_s": round(n / t_dev, 1), "rk_auc_ms": round(1e3 * t_auc, 3),
            "reference_path_ms": round(1e3 * t_ref, 1), "reference_rows_per_s": round(n / t_ref, 1),
            "auc_abs_diff": abs(r[2] - ref[2]), "acc_equal": r[1] == ref[1], "loss_abs_diff": abs(r[0] - ref[0])}


def bench_train(batch, steps, warmup, name="dcn"):
    """Training step (§8(f) #2) at `batch`, wechat tables: zero_grad, forward, the script's loss
    (DCN / DeepCrossing / BST BCEWithLogits on the logit, DIN BCE + l2_reg, the others BCE on the
    probability),
    loss.backward() (HIP backward kernels), Adam step — the reference's train() loop body
    (dcn.py:195-201, deepfm.py:166-171, din.py:339-347, afm.py:168-176, bst.py:276-284,
    fwfm.py:150-157) with the per-call H2 draws frozen; inputs in HBM.  Timed eagerly
    (rankops.Adam) and as one captured hipGraph per step (rankops.Adam(capturable=True))."""
    import helpers as H
    import rankops
    cfg = {"dcn": {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"},
           "deepcrossing": {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"},
           "deepfm": {"vocab": H.WECHAT_VOCAB},
           "din": {"vocab": H.WECHAT_VOCAB, "T": 50, "dim": 32, "interaction_weights": "frozen"},
           "afm": {"vocab": H.WECHAT_VOCAB, "dim": 8, "att": 128},
           "bst": {"vocab": H.WECHAT_VOCAB, "T": 64, "dim": 128, "heads": 4, "max_len": 64},
           "fwfm": {"vocab": H.WECHAT_VOCAB, "dim": 8}}[name]
    inp = None
    res = {"model": {"dcn": "DCN", "deepcrossing": "DeepCrossing", "deepfm": "DeepFM", "din": "DIN", "afm": "AFM",
                     "bst": "BST", "fwfm": "FwFM"}[name], "batch": batch, "config": {k: v for k, v in cfg.items()
                                                                                   if k != "vocab"}}
    on_logit = name in ("dcn", "deepcrossing", "bst")  # BCEWithLogitsLoss (dcn.py:274, deepcrossing.py:256, bst.py:351)
    crit = torch.nn.BCEWithLogitsLoss() if on_logit else torch.nn.BCELoss()
    for mode in ("eager", "graph"):
        torch.manual_seed(0)
        model = H.build(name, cfg).cuda().train()
        if inp is None:
            inp = H.to_device(H.make_inputs(name, cfg, batch, seed=77), "cuda")
            label = (torch.rand(batch, device="cuda") < 0.3).float()
        opt = rankops.Adam(model.parameters(), lr=1e-3, capturable=(mode == "graph"))

        def step():
            opt.zero_grad(set_to_none=True)
            out = H.as_tuple(H.call_model(model, name, inp))
            loss = crit(out[1].squeeze(), label) if on_logit else crit(out[0].squeeze(), label)
            if name == "din":  # ce_loss + l2_reg (din.py:343-344)
                loss = loss + out[2]
            loss.backward()
            opt.step()

        run = step
        if mode == "graph":
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                step()
            run = g.replay
        for _ in range(warmup):
            run()
        torch.cuda.synchronize()
        # best of 3 windows: the eager step is host-bound, and the host is shared with other work
        # on the box (the spread between windows is reported)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(steps):
                run()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / steps)
        t = min(ts)
        res[mode] = {"samples_per_s": round(batch / t, 1), "ms_per_step": round(1e3 * t, 4),
                     "windows_ms": [round(1e3 * x, 4) for x in ts]}
        res["params"] = sum(p.numel() for p in model.parameters())
        del model, opt
    res["eager_over_graph"] = round(res["eager"]["ms_per_step"] / res["graph"]["ms_per_step"], 2)
    res["mode"] = ("forward + loss.backward() + Adam over all params (dense embedding gradients, as "
                   "nn.Embedding(sparse=False) + torch.optim.Adam do)")
    return res


# ------------------------------------------------------------------ embedding-gather roofline (DeepFM configs[1])

def gather_roofline(model, inp, cfg, batch, big_batch=65536):
    """rk_fm_gather alone (30 second-order rows of 128 B + 30 first-order weights + 30 indices read,
    the 3,840-B deep-input row + fm1/fm2 written per sample: 8,048 algorithmic B) over configs[1]'s
    30 x 1e6-row tables, timed with HIP events around hipGraph replays of back-to-back launches
    (graph_kernel_avg_ms: host launch cost excluded), at the config's batch and at 65,536 (steady
    state).  The primary legs read the nn.Embedding weights as they are ([V, 32] rows, one 128-B line
    each, and the [V, 1] first-order table): fm_gather_kernel (sample-major) at 4,096,
    fm_gather_fmaj_kernel (field-major, round 6) from 16,384.  `packed_*`: the rk_fm_pack_table
    layout (one [V, 36] row per index: two 128-B lines), kept for comparison."""
    import helpers as H
    out = {"kernel": "fm_gather_kernel<8, kFmPacked> (4,096) / fm_gather_fmaj_kernel<8, kFmPacked, 6, nt> (65,536)",
           "bound": "hbm", "peak": PEAK_HBM / 1e9, "unit": "GB/s", "bytes_per_sample": DEEPFM_GATHER_BYTES,
           "tables": "30 fields x 1,000,000 rows x 32 fp32 (3.84 GB) + 30 x 1e6 x 1 (beyond the 256 MiB MALL)"}
    dev = torch.device("cuda", torch.cuda.current_device())
    legs = [(f"batch_{batch}", batch, inp["category"]),
            (f"batch_{big_batch}", big_batch, H.to_device(H.make_inputs("deepfm", cfg, big_batch, seed=1234),
                                                          dev)["category"])]
    for b in (batch, big_batch):  # SURVEY §8d cache-sensitivity variant: Zipf(1.1) row popularity
        legs.append((f"zipf_{ZIPF_A}_batch_{b}", b,
                     H.to_device(H.make_inputs("deepfm", dict(cfg, zipf=ZIPF_A), b, seed=4321 + b), dev)["category"]))
    legs += [(f"packed_batch_{b}", b, c) for (_, b, c) in legs[:2]]
    for key, b, cat in legs:
        packed = key.startswith("packed")
        ms = graph_kernel_avg_ms(model.gather_launcher(cat, packed=packed))
        achieved = DEEPFM_GATHER_BYTES * b / (ms * 1e-3)
        # (tools/sessions/r06_counters.sh: workloads deepfm_gather_tables / deepfm_gather at 4,096 and 65,536)
        wl = ("deepfm_gather" if packed else "deepfm_gather_tables") + ("" if b == batch else str(b))
        kern = "fm_gather_fmaj_kernel" if b >= 16384 else "fm_gather_kernel"
        tr = load_traffic(kern, wl) if not key.startswith("zipf") else None
        out[key] = {"avg_launch_ms": round(ms, 5), "achieved": round(achieved / 1e9, 1),
                    "frac": round(achieved / PEAK_HBM, 4), "traffic": tr}
        if tr:  # PMC-measured HBM bytes (2 x FETCH_SIZE + WRITE_SIZE: every L2 read request is 128 B)
            out[key]["hbm_gb_per_s"] = round(tr["bytes_per_launch"] / (ms * 1e-3) / 1e9, 1)
            out[key]["hbm_frac"] = round(tr["bytes_per_launch"] / (ms * 1e-3) / PEAK_HBM, 4)
    return out


# ------------------------------------------------------------------ DCN / BST kernel rooflines

DCN_EXEC_FLOP = 2 * (64 * 512 + 512 * 256 + 256 * 128 + 128) + 3 * 4 * 50  # padded MLP widths + head + cross


def dcn_roofline(model, inp, batch):
    """dcn_fused_kernel (the whole DCN forward, one launch): 20 back-to-back forwards captured in
    one hipGraph, HIP events on the replay stream (the ~1.5 us dependent-launch boundary included)."""
    import helpers as H
    ms = graph_kernel_avg_ms(lambda: H.call_model(model, "dcn", inp))
    flop = DCN_FLOP * batch
    r = {"kernel": "dcn_fused_kernel<1, StreamPlan<4,32,16,8>>", "bound": "mfma", "unit": "TFLOP/s",
         "peak": PEAK_FP32_MFMA / 1e12, "avg_launch_ms": round(ms, 5), "flop_per_launch": flop,
         "flop_basis": "reference formulation per sample: 379,236 (cross 3 x 4 x 50 + 50->512->256->128->1 MLP, "
                       "SURVEY §8d)",
         "achieved": round(flop / (ms * 1e-3) / 1e12, 3), "frac": round(flop / (ms * 1e-3) / PEAK_FP32_MFMA, 4),
         "executed_flop_per_launch": DCN_EXEC_FLOP * batch,
         "frac_executed": round(DCN_EXEC_FLOP * batch / (ms * 1e-3) / PEAK_FP32_MFMA, 4)}
    r.update(counter_fields("dcn_fused_kernel", "dcn", flop))
    return r


DEEPFM_FLOP = 1_310_976  # 960->512->256->128->1 (+ the FM sums' 2 x 960 + final 3 -> 1), SURVEY §8d


def deepfm_roofline(model, inp, batch):
    """deepfm_fused_kernel (the whole DeepFM forward, one launch, rk_deepfm_forward): 20 back-to-back
    forwards captured in one hipGraph, HIP events on the replay stream."""
    import helpers as H
    ms = graph_kernel_avg_ms(lambda: H.call_model(model, "deepfm", inp))
    flop = DEEPFM_FLOP * batch
    r = {"kernel": "deepfm_fused_kernel<StreamPlan<60,32,16,8>>", "bound": "mfma", "unit": "TFLOP/s",
         "peak": PEAK_FP32_MFMA / 1e12, "avg_launch_ms": round(ms, 5), "flop_per_launch": flop,
         "flop_basis": "reference formulation per sample: 1,310,976 (30 x 32 -> 512 -> 256 -> 128 -> 1 deep layers; "
                       "every width a multiple of 64, so also the executed count; SURVEY §8d)",
         "achieved": round(flop / (ms * 1e-3) / 1e12, 3), "frac": round(flop / (ms * 1e-3) / PEAK_FP32_MFMA, 4)}
    r.update(counter_fields("deepfm_fused_kernel", "deepfm", flop))
    return r


def bst_small_roofline(model, inp, batch, cfg):
    """The blocks + pooling of BST at the reference's own shape (d_model 16, one launch) timed alone:
    back-to-back launches, HIP events on the stream they run on.  4 heads: bst_mfma_kernel (round 5:
    projections on v_mfma_f32_16x16x4_f32, QK^T and P V on v_mfma_f32_4x4x1f32, key tiles past each
    sample's length skipped), priced against the FP32 MFMA peak; other head counts: the VALU kernel
    bst_small_kernel.  The flop basis is the reference formulation's (every key position counted)."""
    launch = model.blocks_kernel_launcher(inp["seq_feedid"], inp["seq_length"])
    ms = kernel_avg_ms(launch, 20)
    T, d = cfg["max_len"], cfg["dim"]
    per = 8 * T * d * d + 4 * T * T * d + 4 * T * d * d  # projections, QK^T + AV, FFN (as BST_BLOCK_FLOP)
    nb = len(getattr(model, "transformer_blocks", [None]))
    flop = per * nb * batch
    mfma = cfg.get("heads", 4) == 4 and os.environ.get("RANKOPS_BST_MFMA", "1") != "0"
    r = {"kernel": "bst_mfma_kernel" if mfma else "bst_small_kernel", "bound": "mfma" if mfma else "valu",
         "unit": "TFLOP/s", "peak": PEAK_FP32_MFMA / 1e12,
         "avg_launch_ms": round(ms, 5), "flop_per_launch": flop,
         "flop_basis": f"{per:,} per sample per block (T = {T}, d_model {d}) x {nb} block(s)",
         "achieved": round(flop / (ms * 1e-3) / 1e12, 3), "frac": round(flop / (ms * 1e-3) / PEAK_FP32_MFMA, 4),
         "frac_of_one_wave_valu_issue_peak": round(2 * flop / (ms * 1e-3) / PEAK_FP32_MFMA, 4)}
    if mfma:
        r.update(counter_fields("bst_mfma_kernel", "bst_ref_blocks", flop))
        whole = counter_fields("bst_mfma_fwd_kernel", "bst_ref")
        r["whole_forward_counters"] = {"kernel": "bst_mfma_fwd_kernel", "mfma_busy_frac": whole.get("mfma_busy_frac"),
                                       "counters": whole.get("counters")}
    else:
        r.update(counter_fields("bst_small_kernel", "bst_ref", flop))
    return r


def bst_roofline(model, inp, batch):
    """bst_block_kernel (every transformer block + pooling of the BST forward, one launch) timed
    alone: back-to-back launches, HIP events on the stream they run on."""
    launch = model.blocks_kernel_launcher(inp["seq_feedid"], inp["seq_length"])
    ms = kernel_avg_ms(launch, 20)
    flop = BST_BLOCK_FLOP * batch
    r = {"kernel": "bst_block_kernel", "bound": "mfma", "unit": "TFLOP/s", "peak": PEAK_FP32_MFMA / 1e12,
         "avg_launch_ms": round(ms, 5), "flop_per_launch": flop,
         "flop_basis": "14,680,064 per sample per block: QKV/O projections, QK^T and AV over T = 64, FFN "
                       "(d_model 128, 4 heads; SURVEY §8d)",
         "achieved": round(flop / (ms * 1e-3) / 1e12, 3), "frac": round(flop / (ms * 1e-3) / PEAK_FP32_MFMA, 4)}
    r.update(counter_fields("bst_block_kernel", "bst", flop))
    return r


# AFM forward (afm.py:92-119, D 8, A 128, 7 fields = 21 pairs): per pair the Hadamard product, the
# attention MLP 8 -> 128 (ReLU) -> 1, the softmax-weighted sum; then p (8 -> 1) and the dense term
AFM_FLOP = 21 * (8 + 2 * 8 * 128 + 128 + 2 * 128 + 1) + 21 * 8 * 2 + (2 * 8 + 1) + (2 * 16 + 1)  # 51,647
AFM_BYTES = 7 * (8 + 8 * 4) + 16 * 4 + 2 * 4  # indices + 32-B rows, 16 dense floats, prob + logit: 352
# DeepCrossing forward (deepcrossing.py:146-163, one residual unit 50 -> 128 -> 50, output 50 -> 1)
DEEPCROSSING_FLOP = 2 * 50 * 128 + 128 + 2 * 128 * 50 + 50 + 50 + 2 * 50 + 1  # 25,929
DEEPCROSSING_BYTES = 16 * 4 + 6 * 8 + (16 + 2 + 4 * 4) * 4 + 2 * 4  # dense, 6 indices, 34 embedding floats, outputs: 256


def small_forward_roofline(model, name, inp, batch, flop_per_sample, bytes_per_sample, kernels, big_batch=65536):
    """AFM / DeepCrossing forward legs: the whole eval forward (AFM: one rk_afm_forward
    launch; DeepCrossing: one rk_mlp_forward_gather launch) timed as 20 back-to-back
    forwards in one hipGraph (HIP events on the replay stream), at the bench batch and at 65,536 rows
    (launch ramp amortised).  Both roofs are reported: FP32 matrix/vector peak for the flops, HBM for
    the bytes; at these per-sample sizes neither is close — the forwards are launch- and latency-bound."""
    import helpers as H
    dev = torch.device("cuda", torch.cuda.current_device())
    out = {"kernels": kernels, "flop_per_sample": flop_per_sample, "bytes_per_sample": bytes_per_sample,
           "peak_tflops": PEAK_FP32_MFMA / 1e12, "peak_hbm_gbs": PEAK_HBM / 1e9}
    cfg = workload_cfg(name)
    for b in (batch, big_batch):
        x = inp if b == batch else H.to_device(H.make_inputs(name, cfg, b, seed=4242), dev)
        ms = graph_kernel_avg_ms(lambda x=x: H.call_model(model, name, x))
        out[f"batch_{b}"] = {"avg_forward_ms": round(ms, 5), "samples_per_s": round(b / (ms * 1e-3), 1),
                             "tflops": round(flop_per_sample * b / (ms * 1e-3) / 1e12, 3),
                             "frac_flop": round(flop_per_sample * b / (ms * 1e-3) / PEAK_FP32_MFMA, 4),
                             "gb_per_s": round(bytes_per_sample * b / (ms * 1e-3) / 1e9, 1),
                             "frac_hbm": round(bytes_per_sample * b / (ms * 1e-3) / PEAK_HBM, 4)}
    return out


def workload_cfg(name):
    import helpers as H
    return {"afm": {"vocab": H.WECHAT_VOCAB, "dim": 8, "att": 128},
            "deepcrossing": {"vocab": H.WECHAT_VOCAB, "internal": 128, "units": 1,
                             "interaction_weights": "frozen"}}[name]


# ------------------------------------------------------------------ the driver's line

FINAL_LINE_MAX = 8192  # the driver parses the last stdout line out of a tail of ~8 KB
DEFAULT_DETAILS = os.path.join("gpurun_out", "bench_details.json")


def _frac_of(leg: dict):
    r = leg.get("roofline") or {}
    if "frac" in r:
        return r["frac"]
    b = r.get("batch_4096") or {}
    return b.get("frac_flop")


def models_summary(models: dict) -> dict:
    """Per extra model leg: samples/s, ms per step and (where it has one) the roofline fraction."""
    out = {}
    for k, v in (models or {}).items():
        if not isinstance(v, dict) or "samples_per_s" not in v:
            continue
        e = {"sps": v["samples_per_s"], "ms": v.get("ms_per_step")}
        f = _frac_of(v)
        if f is not None:
            e["frac"] = f
        if k == "deepfm" and isinstance(v.get("gather_roofline"), dict):
            g = v["gather_roofline"]
            e["gather_frac"] = {kk: g[kk]["frac"] for kk in g if isinstance(g[kk], dict) and "frac" in g[kk]}
        out[k] = e
    return out


def compact_result(full: dict, details_path: str = None) -> dict:
    """The driver's line: the contract keys, `roofline` with a numeric `traffic`, `cpu_baseline` with
    its legs reduced to {value, cores, gpu_over_cpu}, and one-line summaries of the extra legs; the
    full result (every leg's detail) is in `details_path` (bench_details.json)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "build")
    out = {k: full[k] for k in keep if k in full}
    r = full.get("roofline")
    if r:
        tr = r.get("traffic")
        ctr = r.get("counters") or {}
        out["roofline"] = {
            "kernel": r["kernel"], "bound": r["bound"], "achieved": r["achieved"], "peak": r["peak"],
            "unit": r["unit"], "frac": r["frac"],
            "traffic": tr["bytes_per_launch"] if isinstance(tr, dict) else tr,
            "avg_launch_ms": r.get("avg_launch_ms"), "flop_per_launch": r.get("flop_per_launch"),
            "flop_basis": "reference formulation, SURVEY §8d (1,478,272 flop/sample)",
            "frac_executed": r.get("frac_executed"), "mfma_busy_frac": r.get("mfma_busy_frac"),
            "counters": {"session": ctr.get("session"), "staleness": ctr.get("staleness"),
                         "traffic_session": tr.get("session") if isinstance(tr, dict) else None,
                         "traffic_staleness": tr.get("staleness") if isinstance(tr, dict) else None,
                         "file": COUNTERS_FILE}}
    cb = full.get("cpu_baseline")
    if cb:
        c = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample", "gpu_over_cpu") if k in cb}
        c["legs"] = {k: {kk: v[kk] for kk in ("value", "cores", "gpu_over_cpu") if kk in v}
                     for k, v in (cb.get("legs") or {}).items()}
        out["cpu_baseline"] = c
    if full.get("models"):
        out["models"] = models_summary(full["models"])
    sh = full.get("sharded_deepfm")
    if isinstance(sh, dict):
        s = {k: sh[k] for k in ("samples_per_s", "ms_per_step", "scaling", "wire_format", "error") if k in sh}
        mc = (sh.get("model_curve") or {}).get("curve")
        if mc:
            s["model_speedup_pipelined"] = {p: (v.get("speedup_vs_p1") or {}).get("pipelined")
                                            for p, v in mc.items() if p != "1"}
        out["sharded_deepfm"] = s
    if details_path:
        out["details"] = details_path
    return out


def emit(result: dict, details_path: str):
    """Write the full result to `details_path`, print a summary of the extras, then the compact
    line last (asserted under FINAL_LINE_MAX bytes)."""
    if details_path:
        os.makedirs(os.path.dirname(os.path.abspath(details_path)), exist_ok=True)
        with open(details_path, "w") as f:
            json.dump(result, f, indent=1)
    line = json.dumps(compact_result(result, details_path))
    if len(line.encode()) > FINAL_LINE_MAX:  # never let the headline grow past what the driver parses
        slim = compact_result({k: v for k, v in result.items() if k not in ("models", "sharded_deepfm")},
                              details_path)
        line = json.dumps(slim)
    print(line, flush=True)


# ------------------------------------------------------------------ main

def bench_one(name, batch, steps, warmup, world, rank, zipf=None, streams=1):
    model, inp, fn, cfg, model_name = workload(name, batch, rank, zipf)
    if name.endswith("per_call") or name.endswith("_eager"):
        # eager: one Python forward per step, as the reference's evaluate() / predict loops call
        # the model (dcn.py:214-239); per-call H2 draws + H2D included in the per_call legs
        def run():
            with torch.no_grad():
                fn()
        n = max(20, steps // 2) if name.endswith("per_call") else steps
        t = time_replays(run, n, 5 if name.endswith("per_call") else warmup, 1)
        mode = "eager, per-call H2 draws" if name.endswith("per_call") else "eager (no graph), frozen H2"
        return {"samples_per_s": round(batch * n / t, 1), "mode": mode,
                "ms_per_step": round(1e3 * t / n, 4)}, model, inp, cfg, model_name
    g, _ = graph_of(fn)
    res = {}
    if model_name == "din":
        # the whole DIN forward is one kernel: a prepared launch (DIN.prepare ->
        # rk_din_forward_plan) replays it without a graph's per-replay gap; the graph replay of the
        # same forward is timed too and reported beside it
        run = model.prepare(inp["dense"], inp["category"], inp["sequence"], inp["target"])
        tg = max_over_ranks(world, time_replays(g.replay, steps, warmup, world))
        res["graph_replay_ms_per_step"] = round(1e3 * tg / steps, 4)
        res["step"] = "prepared single-kernel launch (rk_din_plan_launch)"
        if streams > 1:
            # S batches in flight: S prepared launches, each with its own inputs (seeded apart),
            # outputs and l2 workspace, issued round-robin on S HIP streams, so the next batch's
            # workgroups take the CUs the previous batch's tail frees (tools/din_streams.py:
            # outputs bit-identical to single-stream launches).  Every step is still one whole
            # batch forward, all of them inside the timed window.
            import helpers as H
            t1 = max_over_ranks(world, time_replays(run, steps, warmup, world))
            res["single_stream_samples_per_s"] = round(world * batch * steps / t1, 1)
            res["single_stream_ms_per_step"] = round(1e3 * t1 / steps, 4)
            dev = torch.device("cuda", torch.cuda.current_device())
            runs = [run]
            for i in range(1, streams):
                x = H.to_device(H.make_inputs(model_name, cfg, batch, seed=1000 + rank + 7919 * i), dev)
                runs.append(model.prepare(x["dense"], x["category"], x["sequence"], x["target"]))
            strs = [torch.cuda.Stream() for _ in range(streams)]
            for st in strs:
                st.wait_stream(torch.cuda.current_stream())
            plans = [r.plan for r in runs]
            handles = [st.cuda_stream for st in strs]
            cnt = [0]

            def run():
                i = cnt[0] % streams
                cnt[0] += 1
                plans[i].launch_on(handles[i])
            res["step"] = (f"prepared single-kernel launches (rk_din_plan_launch), {streams} batches in flight "
                           f"on {streams} HIP streams (round-robin, own inputs/outputs/workspaces)")
    elif model_name in ("dcn", "deepfm") and not zipf:
        # DCN and (at configs[1]'s shape) DeepFM are single-kernel forwards too: a prepared launch
        # (DCNModel.prepare / DeepFM.prepare: the cached ctypes call of rk_dcn_forward /
        # rk_deepfm_forward bound to the inputs), the graph replay of the same forward beside it
        run = model.prepare(inp["dense"], inp["category"]) if model_name == "dcn" else model.prepare(inp["category"])
        tg = max_over_ranks(world, time_replays(g.replay, steps, warmup, world))
        res["graph_replay_ms_per_step"] = round(1e3 * tg / steps, 4)
        res["step"] = "prepared launch (%s)" % ("rk_dcn_forward" if model_name == "dcn" else "rk_deepfm_forward")
    elif name == "afm":
        # one kernel (rk_afm_forward): AFM.prepare binds it to the inputs; graph replay beside it
        run = model.prepare(inp["dense_input"], inp["category_input"])
        tg = max_over_ranks(world, time_replays(g.replay, steps, warmup, world))
        res["graph_replay_ms_per_step"] = round(1e3 * tg / steps, 4)
        res["step"] = "prepared launch (rk_afm_forward)"
    elif name == "deepcrossing":
        # the row gather and the residual MLP in one launch, bound to the inputs (DeepCrossingModel.prepare)
        run = model.prepare(inp["dense"], inp["category"])
        tg = max_over_ranks(world, time_replays(g.replay, steps, warmup, world))
        res["graph_replay_ms_per_step"] = round(1e3 * tg / steps, 4)
        res["step"] = "prepared launch (rk_mlp_forward_gather)"
    elif name == "fwfm":
        # one kernel (rk_fwfm_forward): FwFM.prepare binds it to the inputs; graph replay beside it
        run = model.prepare(inp["x"])
        tg = max_over_ranks(world, time_replays(g.replay, steps, warmup, world))
        res["graph_replay_ms_per_step"] = round(1e3 * tg / steps, 4)
        res["step"] = "prepared launch (rk_fwfm_forward)"
    elif name == "bst_ref":
        # at the reference script's d_model 16 the whole BST forward is one kernel too
        # (rk_bst_small_forward): BSTModel.prepare binds it to the inputs; graph replay beside it
        run = model.prepare(inp["dense"], inp["category"], inp["seq_feedid"], inp["seq_length"])
        tg = max_over_ranks(world, time_replays(g.replay, steps, warmup, world))
        res["graph_replay_ms_per_step"] = round(1e3 * tg / steps, 4)
        res["step"] = "prepared launch (rk_bst_small_forward)"
    else:
        run = g.replay
    t = time_replays(run, steps, warmup, world)
    t = max_over_ranks(world, t)
    res.update({"samples_per_s": round(world * batch * steps / t, 1), "ms_per_step": round(1e3 * t / steps, 4)})
    if zipf is not None:
        res["index_distribution"] = f"Zipf({zipf}) over table rows (hot rows scattered)"
    return res, model, inp, cfg, model_name


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    import rankops
    rankops.load_library()
    torch.backends.cuda.matmul.allow_tf32 = False

    head, model, inp, cfg, model_name = bench_one("din", args.batch, args.steps, args.warmup, world, rank,
                                                  streams=args.din_streams)
    result = {
        "metric": METRIC,
        "value": head["samples_per_s"],
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded wechat-shaped ids, log1p(Poisson(2)) dense, random-init weights)",
        "config": {"workload": "configs[2]: DIN forward, seq_len 50, emb_dim 32, batch 4096 per GPU",
                   "model": "DIN", "global_batch": world * args.batch, "seq_len": 50, "emb_dim": 32,
                   "tables": "wechat_algo_data1 sizes (feedid 106445 rows)", "mode": "eval, inputs resident in HBM",
                   "interaction_weights": "frozen", "parallelism": f"replicas x{world}",
                   "step": head.get("step"), "graph_replay_ms_per_step": head.get("graph_replay_ms_per_step"),
                   "single_stream_samples_per_s": head.get("single_stream_samples_per_s"),
                   "single_stream_ms_per_step": head.get("single_stream_ms_per_step")},
    }
    from rankops import _lib as rk_lib
    bi = rk_lib.build_info()
    global _LIB_SRC
    _LIB_SRC = bi.get("src")
    result["build"] = {"lib_src_hash": bi.get("src"), "tree_src_hash": bi.get("tree_src"), "arch": bi.get("arch"),
                       "extra_flags": bi.get("extra"),
                       "lib_matches_tree": bi.get("tree_src") is not None and bi.get("src") == bi.get("tree_src")}
    if rank == 0:
        # the kernel the headline times: a prepared plan's launch (rk_din_plan_launch, host cost a
        # few us against the ~44-us kernel, so back-to-back launches keep the GPU busy)
        launch = model.prepare(inp["dense"], inp["category"], inp["sequence"], inp["target"]).plan.launch
        ms = kernel_avg_ms(launch)
        flop = DIN_FWD_FLOP * args.batch
        achieved = flop / (ms * 1e-3)
        result["roofline"] = {"kernel": "din_forward_kernel<32>", "bound": "mfma",
                              "achieved": round(achieved / 1e12, 3), "peak": PEAK_FP32_MFMA / 1e12,
                              "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_MFMA, 4),
                              "avg_launch_ms": round(ms, 5), "flop_per_launch": flop,
                              "flop_basis": "reference formulation per sample: att-MLP 1,027,200 + cross/"
                                            "weighted sum 6,400 + fcn 444,672 (SURVEY §8d)",
                              "executed_flop_per_launch": DIN_FWD_EXEC_FLOP * args.batch,
                              "frac_executed": round(DIN_FWD_EXEC_FLOP * args.batch / (ms * 1e-3) / PEAK_FP32_MFMA, 4),
                              "traffic": load_traffic("din_forward_kernel", "din")}
        result["roofline"].update(counter_fields("din_forward_kernel", "din", flop))
    if rank == 0 and world == 1 and not args.no_extras:
        extras = {}
        for name in [m for m in args.models.split(",") if m]:
            batch = {"bst": 2048, "bst_eager": 2048, "dcn_256_per_call": 256}.get(name, args.batch)
            zipf = ZIPF_A if name.endswith("_zipf") else None
            r, m2, inp2, cfg2, mn2 = bench_one(name[:-5] if zipf else name, batch, args.steps, args.warmup, 1, 0,
                                               zipf=zipf)
            if name.endswith("_eager") and name[:-6] in extras:
                r["eager_over_graph"] = round(r["ms_per_step"] / extras[name[:-6]]["ms_per_step"], 3)
            if name == "bst":
                r["gflop_per_s_block"] = round(BST_BLOCK_FLOP * r["samples_per_s"] / 1e9, 1)
                r["roofline"] = bst_roofline(m2, inp2, batch)
            if name == "bst_ref":
                r["roofline"] = bst_small_roofline(m2, inp2, batch, cfg2)
            if name == "dcn":
                r["roofline"] = dcn_roofline(m2, inp2, batch)
            if name == "deepfm":
                r["roofline"] = deepfm_roofline(m2, inp2, batch)
            if name == "deepfm":
                r["gather_roofline"] = gather_roofline(m2, inp2, cfg2, batch)
            if name == "afm":
                r["roofline"] = small_forward_roofline(m2, "afm", inp2, batch, AFM_FLOP, AFM_BYTES,
                                                       ["afm_tiles_kernel<2,8,4>"])
                r["roofline"].update(counter_fields("afm_tiles_kernel", "afm"))
            if name == "deepcrossing":
                r["roofline"] = small_forward_roofline(m2, "deepcrossing", inp2, batch, DEEPCROSSING_FLOP,
                                                       DEEPCROSSING_BYTES, ["dc_forward_kernel<8,1>"])
                r["roofline"].update(counter_fields("dc_forward_kernel", "deepcrossing"))
            if name == "fwfm":  # 6 x (8 B index + 32 B embedding row + 4 B linear) + 4 B prob
                r["gather_gb_per_s"] = round(FWFM_BYTES_PER_SAMPLE * r["samples_per_s"] / 1e9, 1)
                r["bytes_per_sample"] = FWFM_BYTES_PER_SAMPLE
                big, mb, _, _, _ = bench_one("fwfm", 1 << 20, max(5, args.steps // 5), 3, 1, 0)
                big["gather_gb_per_s"] = round(FWFM_BYTES_PER_SAMPLE * big["samples_per_s"] / 1e9, 1)
                r["batch_1m"] = big
                del mb
            extras[name] = r
            del m2, inp2
            torch.cuda.empty_cache()
        result["models"] = extras
    if rank == 0 and world == 1 and not args.no_loader:
        try:
            result["loader"] = bench_loader(model, args.batch)
        except Exception as exc:  # reported, never fatal for the headline line
            result["loader"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
    if rank == 0 and world == 1 and not args.no_extras and not args.no_train:
        try:
            result["train"] = {m: bench_train(2048 if m == "bst" else args.batch, max(10, args.steps // 2), 10, m)
                               for m in ("dcn", "deepcrossing", "deepfm", "din", "afm", "bst", "fwfm")}
        except Exception as exc:  # reported, never fatal for the headline line
            result["train"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
    if rank == 0 and world == 1 and not args.no_loader:
        try:
            result["eval_metrics"] = bench_metrics(args.batch)
        except Exception as exc:  # reported, never fatal for the headline line
            result["eval_metrics"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
    if not args.no_sharded:
        torch.cuda.empty_cache()
        try:
            sh = bench_sharded(world, rank, args.steps, args.warmup)
        except Exception as exc:  # reported, never fatal for the headline line
            sh = {"error": f"{type(exc).__name__}: {exc}"[:300]}
        if world == 1 and "ms_per_step" in sh and not args.no_model_curve:
            try:
                sh["model_curve"] = sharded_model_curve(sh["ms_per_step"])
            except Exception as exc:
                sh["model_curve"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
            torch.cuda.empty_cache()
        result["sharded_deepfm"] = sh
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baselines(model.cpu(), cfg, result["value"], result.get("models", {}),
                                               args.batch, args.cpu_seconds)
    if rank == 0:
        emit(result, args.details)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
