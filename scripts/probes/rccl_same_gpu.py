"""Probe: can two RCCL ranks share the one GPU of a gpurun box?

Launched as ``python -m torch.distributed.run --nproc-per-node 2
--master-addr 127.0.0.1 --master-port P scripts/probes/rccl_same_gpu.py``.
Every rank binds cuda:0, initialises the "nccl" (RCCL) backend and runs the
collectives the sharded sweeps use (all_gather_into_tensor, all_reduce MAX,
point-to-point send/recv), checking their results.
"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    n = 1 << 20
    x = torch.full((n,), rank + 1, dtype=torch.uint8, device=dev)
    out = torch.empty(world * n, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, x)
    torch.cuda.synchronize()
    ref = torch.arange(1, world + 1, dtype=torch.uint8, device=dev).repeat_interleave(n)
    ok = bool(torch.equal(out, ref))
    t = torch.tensor([float(rank) * 3.5], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok &= float(t.item()) == (world - 1) * 3.5
    if world > 1:
        if rank == 1:
            dist.send(torch.full((4096,), 7.0, device=dev), dst=0)
        elif rank == 0:
            r = torch.empty(4096, device=dev)
            dist.recv(r, src=1)
            ok &= bool((r == 7.0).all())
    dist.barrier()
    print("rank %d/%d rccl %s ok=%s" % (rank, world, torch.cuda.nccl.version()
                                       if hasattr(torch.cuda, "nccl") else "?", ok), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
