"""The pipelined DM-sharded step's stream ordering with real HIP kernels.

RCCL refuses two ranks on one device ("Duplicate GPU detected",
scripts/probes/rccl_two_ranks.py), so on a one-GPU box the all-gather of
DMShardedSweep is replaced by a loopback with RCCL's semantics: it runs on a
side stream after the rank's corner turn (event), is delayed by a spin kernel
(~20 ms, longer than a batch's sweep here), copies the batch's pieces of
every rank -- its own from the corner-turn buffer -- into the block, and its
wait() makes the compute stream wait for it.  A missing wait (the sweep would
read the stale block, filled with 255) or a corner-turn buffer reused before
the exchange read it (batch k+2's turn overwriting batch k's piece) changes
the plane; both ranks' rows must equal the one-shot plane bit for bit."""
import numpy as np
import pytest

from conftest import band

DT = 64e-6
pytestmark = pytest.mark.gpu


class _Work(object):
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_event(self.ev)


@pytest.mark.parametrize("rank", [0, 1])
def test_pipeline_ordering_with_delayed_loopback_gather(gpu, rank):
    import torch
    from pypulsar_amd.sharding import DMShardedSweep, split_block, trial_work
    from pypulsar_amd.sweep import DMSweep
    C, N, D, W, NB = 1024, 1 << 18, 512, 2, 4
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    g = torch.Generator(device="cuda")
    g.manual_seed(77)
    block = torch.randint(0, 256, (N, C), generator=g, device="cuda", dtype=torch.uint8)
    sw = DMSweep(dms, freqs, DT, dtype="u8")
    plane = sw(block.t().contiguous())
    sw.close()
    P = N // (NB * W)
    remote = torch.empty((N // P, C, P), dtype=torch.uint8, device="cuda")
    for b in range(N // P):
        remote[b].copy_(block[b * P:(b + 1) * P].t())
    side = torch.cuda.Stream()
    calls = []

    def gather_fn(out, cm, k):
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())
        side.wait_event(ready)
        with torch.cuda.stream(side):
            torch.cuda._sleep(50_000_000)          # the exchange lands late
            out.copy_(remote[k * W:(k + 1) * W].reshape(W * C, P))
            out.view(W, C, P)[rank].copy_(cm)     # this rank's own piece: its corner turn
        done = torch.cuda.Event()
        done.record(side)
        calls.append(k)
        return _Work(done)

    ds = DMShardedSweep(dms, freqs, DT, N, dtype=torch.uint8, n_batches=NB,
                        work=trial_work(dms, 1), device="cuda", world=W, rank=rank,
                        gather_fn=gather_fn)
    assert ds.pieces and len(ds.cm) == 2
    part = split_block(block, NB, W, rank)
    for step in range(2):
        ds.x.fill_(255)                            # what a premature sweep would read
        ds(part)
        torch.cuda.synchronize()
        assert torch.equal(ds.plane(), plane[ds.lo:ds.hi]), "step %d" % step
    assert calls == list(range(NB)) * 2
    ds.close()


@pytest.mark.parametrize("world,rank", [(1, 0), (4, 1), (4, 3)])
def test_timeshard_host_step_device_equals_resident(gpu, world, rank):
    """TimeShardedSweep.host_step on the device (the PCIe-inclusive leg of
    bench.py at N > 1): the rank's input spectra in PINNED host memory, 4
    H2D chunks on a copy stream (edges rounded up to 16 spectra) under 4
    column ranges of the factorised 8-bit sweep -- the rank's plane equals
    the resident step (__call__) bit for bit, and (W = 1) the one-shot
    DMSweep plane."""
    import torch
    from pypulsar_amd.sharding import TimeShardedSweep
    from pypulsar_amd.sweep import DMSweep
    C, N, D = 1024, 1 << 18, 512
    freqs = band(C)
    dms = np.linspace(0.0, 1000.0, D)
    g = torch.Generator(device="cuda")
    g.manual_seed(91)
    block = torch.randint(0, 256, (N, C), generator=g, device="cuda", dtype=torch.uint8)
    ts = TimeShardedSweep(dms, freqs, DT, N, dtype=torch.uint8, world=world, rank=rank,
                          device="cuda")
    assert ts.sw.factor_info(1)[0] in (2, 4)
    lo, hi = ts.input_range()
    want = ts(block[lo:hi].contiguous()).clone()
    hpart = torch.empty((hi - lo, C), dtype=torch.uint8, pin_memory=True)
    hpart.copy_(block[lo:hi])
    ts.out.fill_(-1.0)
    got = ts.host_step(hpart, n_batches=4)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    if world == 1:
        sw = DMSweep(dms, freqs, DT, dtype="u8")
        assert torch.equal(want, sw(block.t().contiguous()))
        sw.close()
    ts.close()
