"""In-process all-to-all emulator for the table-sharded DeepFM (rankops.sharded) — test harness.

P ShardedDeepFM shards live in one process, each driven by its own Python thread; every shard's
`exchange_fn` is bound to one InProcessAllToAll.  A call is collective, like
`torch.distributed.all_to_all_single(out, inp, out_splits, in_splits)`: all P ranks deposit their
send buffer, meet at a barrier, each copies the pieces addressed to it (source order, the split
sizes checked against each other), and meet again before anyone may reuse a buffer.  On a GPU the
copies are stream-ordered after the producers (all threads enqueue on the device's default
stream after an event wait on every rank's producers, whatever streams the ranks use), so every
device step of the shards stays real and only the RCCL transport is replaced."""
from __future__ import annotations

import threading


class _Done:
    """Work handle of an exchange whose copies were enqueued at issue time: wait() orders the
    caller's current stream after them (a no-op for CPU tensors), as a ProcessGroupNCCL work's
    wait() does."""

    def __init__(self, event=None):
        self.event = event

    def wait(self):
        if self.event is not None:
            import torch
            torch.cuda.current_stream().wait_event(self.event)
        return True


class InProcessAllToAll:
    def __init__(self, world: int, timeout: float = 120.0):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.slots = [None] * world
        self.events = [None] * world
        self.calls = 0

    def bind(self, rank: int):
        def exchange(out, inp, out_splits, in_splits, async_op=False):
            ev = self._exchange(rank, out, inp, list(out_splits), list(in_splits))
            return (out, _Done(ev)) if async_op else out
        return exchange

    def _exchange(self, rank, out, inp, out_splits, in_splits):
        """Stream-ordered on a GPU: each rank's copies run on its current stream after every
        rank's producers (an event per rank recorded at deposit), and every rank's stream then
        waits for every rank's copies (so no send buffer is reused while a peer still reads it).
        Returns the event after this rank's copies (None on CPU)."""
        import torch
        if len(out_splits) != self.world or len(in_splits) != self.world:
            raise ValueError("split lists must have one entry per rank")
        if sum(in_splits) != inp.numel() or sum(out_splits) != out.numel():
            raise ValueError(f"rank {rank}: split sums {sum(in_splits)}/{sum(out_splits)} != "
                             f"buffer sizes {inp.numel()}/{out.numel()}")
        cuda = out.is_cuda
        self.slots[rank] = (inp.reshape(-1), in_splits)
        if cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self.events[rank] = ev
        self.barrier.wait()
        if cuda:
            st = torch.cuda.current_stream()
            for e in list(self.events):
                st.wait_event(e)
        flat = out.reshape(-1)
        o = 0
        for s in range(self.world):
            src, splits = self.slots[s]
            n = splits[rank]
            if n != out_splits[s]:
                raise ValueError(f"rank {rank} expects {out_splits[s]} elements from {s}, which sends {n}")
            start = sum(splits[:rank])
            flat[o:o + n].copy_(src[start:start + n])
            o += n
        if rank == 0:
            self.calls += 1
        done = None
        self.barrier.wait()  # every rank has read the deposit events
        if cuda:
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream())
            self.events[rank] = done
        self.barrier.wait()
        if cuda:
            st = torch.cuda.current_stream()
            for e in list(self.events):
                st.wait_event(e)
        self.barrier.wait()  # every rank has read the copy events before the next call replaces them
        return done

    def abort(self):
        self.barrier.abort()


def run_ranks(world: int, fn, on_error=None, timeout: float = 300.0):
    """Runs fn(rank) on `world` threads; returns the per-rank results, re-raising the first
    error.  `on_error` (e.g. InProcessAllToAll.abort) runs when a rank fails, so the others stop
    at the barrier instead of waiting for it."""
    results, errors = [None] * world, [None] * world

    def body(r):
        try:
            results[r] = fn(r)
        except BaseException as exc:  # noqa: BLE001 - re-raised in the caller
            errors[r] = exc
            if on_error is not None:
                on_error()

    threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout)
        if t.is_alive():
            raise TimeoutError("emulated rank did not finish")
    real = [e for e in errors if e is not None and not isinstance(e, threading.BrokenBarrierError)]
    if real:
        raise real[0]
    for e in errors:
        if e is not None:
            raise e
    return results
