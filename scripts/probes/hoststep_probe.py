"""TimeShardedSweep.host_step of single ranks of a W = 8 configs[3] split on
one GPU, in a chosen order, with the free device memory, the wall time and
the sweep kernel time / launches of each timed step: why one rank of the
`bench.py --rehearse 8 --mode timeshard` PCIe leg is slower."""
import sys
import time
import numpy as np
import torch
sys.path.insert(0, ".")
import bench
from pypulsar_amd.sharding import TimeShardedSweep

order = [int(r) for r in (sys.argv[1] if len(sys.argv) > 1 else "5,0,5,6").split(",")]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
C, N, D = 4096, 1 << 22, 4096
freqs = bench.band(C)
dms = np.linspace(0.0, 1000.0, D)
block = bench.synth_block(N, C, 1000, "u8", dev)
for r in order:
    ts = TimeShardedSweep(dms, freqs, 64e-6, N, dtype=torch.uint8, world=8, rank=r, device=dev)
    lo, hi = ts.input_range()
    hpart = torch.empty((hi - lo, C), dtype=torch.uint8, pin_memory=True)
    hpart.copy_(block[lo:hi])
    cs = torch.cuda.Stream(device=dev)
    ts.host_step(hpart, n_batches=4, copy_stream=cs)
    torch.cuda.synchronize()
    for it in range(3):
        free = torch.cuda.mem_get_info(dev)[0]
        ts.sw.set_timing(True)
        t0 = time.perf_counter()
        ts.host_step(hpart, n_batches=4, copy_stream=cs)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3
        kms, launches = ts.sw.timing_read()
        ts.sw.set_timing(False)
        print("rank %d it %d: %.1f ms  sweep %.1f ms / %d launches  free %.1f GB  hpart %#x"
              % (r, it, el, kms, launches, free / 1e9, hpart.data_ptr()), flush=True)
    t0 = time.perf_counter()
    ts(block[lo:hi])
    torch.cuda.synchronize()
    print("rank %d resident step %.1f ms" % (r, (time.perf_counter() - t0) * 1e3), flush=True)
    ts.close()
    del ts, hpart
    torch.cuda.empty_cache()
print("probe done")
