"""Probe: can two ranks share one GPU under RCCL (backend "nccl")?  If they
can, DMShardedSweep's pipelined all-gather path (tests/test_gpu_rccl.py) runs
for real with the HIP kernels on a one-GPU box.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 scripts/probes/rccl_two_ranks.py
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
    part = torch.full((4, 1024), float(rank + 1), device=dev)
    out = torch.empty((4 * world, 1024), device=dev)
    w = dist.all_gather_into_tensor(out, part, async_op=True)
    w.wait()
    torch.cuda.synchronize()
    ok = all(float(out[4 * r:4 * r + 4].mean()) == r + 1 for r in range(world))
    print("rank %d: all_gather_into_tensor %s" % (rank, "OK" if ok else "WRONG"), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
