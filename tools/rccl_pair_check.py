"""Can two ranks share one GPU under RCCL (a one-GPU rehearsal of bench.py's N > 1 path)?  RCCL
refuses it ("Duplicate GPU detected", profiles/r05/rccl_pair.log); BACKEND=gloo runs the same
check over gloo with the tensors on the GPU.  Launch:
python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511
tools/rccl_pair_check.py.  Each rank all-to-alls a small tensor and checks what it received."""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    backend = os.environ.get("BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(backend)
    send = torch.arange(world * 4, device="cuda", dtype=torch.float32) + 100 * rank
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    torch.cuda.synchronize()
    want = torch.cat([torch.arange(4, device="cuda", dtype=torch.float32) + 4 * rank + 100 * s for s in range(world)])
    t = torch.tensor([float(rank)], device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    print(f"rank {rank} on cuda:{dev} ({backend}): all_reduce max {t.item()}, all_to_all_single {'ok' if torch.equal(recv, want) else 'WRONG'} {recv.tolist()}",
          flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
