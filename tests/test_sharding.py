"""Multi-rank paths on CPU: world_size-2 (and 3) gloo process groups running
the same partition / broadcast / gather code the GPU box runs over RCCL.
The per-rank compute is the oracle sweep here (injected); on the GPU it is
the HIP DMSweep."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pypulsar_amd import sharding

DT = 64e-6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _band(C):
    foff = -300.0 / C
    return 1550.0 + foff / 2 + foff * np.arange(C)


def _data(C, N):
    rng = np.random.default_rng(3)
    return np.clip(np.round(rng.normal(128, 16, (C, N))), 0, 255).astype(np.float32)


def _oracle_sweep(freqs, n_out):
    from oracle import spectra_oracle as orc

    def fn(x, dms):
        tab = orc.sweep_table(dms, freqs, DT)
        return torch.from_numpy(orc.sweep_plane(x.numpy().astype(np.float64), tab, n_out=n_out)
                                .astype(np.float32))
    return fn


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        C, N, NB, NBP = 16, 1000, 2400, 4096
        freqs = _band(C)
        dms = np.linspace(0.0, 40.0, 11)
        from oracle import spectra_oracle as orc
        n_out = N - int(orc.sweep_table(dms, freqs, DT).max())
        x = torch.from_numpy(_data(C, N)) if rank == 0 else None
        plane = sharding.dm_sharded_sweep(x, (C, N), torch.float32, dms, freqs, DT, n_out,
                                          sweep_fn=_oracle_sweep(freqs, n_out), src=0, dst=0)
        # time-block shards: each rank its own output range, no collective
        tab = orc.sweep_table(dms, freqs, DT)
        lo, hi, ilo, ihi = sharding.timeblock_ranges(n_out, world, tab.max())[rank]
        xb = _data(C, N)[:, ilo:min(ihi, N)].astype(np.float64)
        part = orc.sweep_plane(xb, tab, n_out=hi - lo)
        parts = [None] * world
        dist.all_gather_object(parts, part)
        # DM-sharded sweep + local search: only candidates are exchanged
        from oracle import search_oracle as so
        from pypulsar_amd.search import to_records
        xs = _data(C, N)
        xs[:, 300:304] += 60.0  # undispersed burst: strongest near DM 0
        xs = torch.from_numpy(xs) if rank == 0 else None

        def search_fn(plane, sub):
            c, _ = so.search(plane.numpy().astype(np.float64), (1, 2, 4, 8), 5.0, 200)
            raw = np.array([(d, t, w, np.float32(s).view(np.int32)) for d, t, w, s in c],
                           dtype=np.int32).reshape(-1, 4)
            return to_records(raw, sub, DT)
        cands = sharding.dm_sharded_search(xs, (C, N), torch.float32, dms, freqs, DT, n_out,
                                           sweep_fn=_oracle_sweep(freqs, n_out),
                                           search_fn=search_fn)
        # pipelined DM sharding (DMShardedSweep): per-rank H2D slices of every
        # time batch, all-gathered batch by batch; planes resident (ag) or
        # gathered to rank 0 batch by batch (agg); DM slices work-weighted
        work = np.r_[np.ones(5), np.full(len(dms) - 5, 0.5)]

        def to_cm(src_tc, dst_cm):
            dst_cm.copy_(src_tc.t())

        def sweep_fn(x, N, piece, x_off, sub, out, n_cols):
            if piece:  # [N/P][C][P] pieces -> channel-major
                x = x.reshape(N // piece, C, piece).permute(1, 0, 2).reshape(C, N)
            tab = orc.sweep_table(sub, freqs, DT)
            xv = x[:, x_off:x_off + n_cols + int(tab.max())]
            out.copy_(torch.from_numpy(orc.sweep_plane(xv.numpy().astype(np.float64), tab,
                                                       n_out=n_cols).astype(np.float32)))
        # time sharding (TimeShardedSweep): rank r sweeps plane columns
        # [a_r, b_r) of the whole grid from its own input spectra, no
        # collective; resident blocks, or gathered to rank 0
        def ts_sweep(x, out, n_cols):
            tab = orc.sweep_table(dms, freqs, DT)
            out.copy_(torch.from_numpy(orc.sweep_plane(x.numpy().astype(np.float64), tab,
                                                       n_out=n_cols).astype(np.float32)))
        blk = torch.from_numpy(_data(C, NB).T.copy())
        ts_res = {}
        for gather in (False, True):
            ts = sharding.TimeShardedSweep(dms, freqs, DT, NB, dtype=torch.float32, gather=gather,
                                           to_cm=to_cm, sweep_fn=ts_sweep, align=64)
            lo, hi = ts.input_range()
            for _ in range(2):
                out = ts(blk[lo:hi].contiguous())
            ts_res[gather] = (ts.a, out.numpy().copy())
            # the PCIe-inclusive step (bench.py's end_to_end_pcie leg at N > 1),
            # with and without the gather to rank 0: the same result
            ts_res[("host", gather)] = ts.host_step(blk[lo:hi].contiguous(), n_batches=3).numpy().copy()
        tsr = [None] * world
        dist.all_gather_object(tsr, ts_res[False])
        res = {}
        # NB = 2400 splits into 2 batches x world slices of 600 or 400 spectra
        # (time-major path); NBP = 4096 into power-of-two slices (pieces path)
        cases = [(False, NB, False), (True, NB, False)]
        if world in (1, 2, 4, 8):  # power-of-two slices of NBP: the pieces path
            cases += [(False, NBP, True), (True, NBP, True)]
        for gather, nbk, pieces in cases:
            xs = torch.from_numpy(_data(C, nbk).T.copy())
            ds = sharding.DMShardedSweep(dms, freqs, DT, nbk, dtype=torch.float32, n_batches=2,
                                         work=work, gather=gather, to_cm=to_cm,
                                         sweep_fn=sweep_fn)
            assert ds.pieces == pieces
            part = sharding.split_block(xs, 2, world, rank)
            for _ in range(2):  # a second step reuses every buffer
                ds(part)
            res[(gather, pieces)] = (ds.lo, ds.hi, ds.plane().numpy(), ds.slices)
        ag = [None] * world
        dist.all_gather_object(ag, res[(False, False)][:3])
        agp = [None] * world
        dist.all_gather_object(agp, res.get((False, True), (0, 0, None))[:3])
        # plane gather into a preallocated plane (no concatenation)
        g = sharding.gather_planes(torch.from_numpy(res[(False, False)][2]), res[(False, False)][3])
        if rank == 0:
            q.put(("ag", np.concatenate([p for _, _, p in sorted(ag, key=lambda a: a[0])])))
            q.put(("agg", res[(True, False)][2]))
            if (False, True) in res:
                q.put(("agp", np.concatenate([p for _, _, p in sorted(agp, key=lambda a: a[0])])))
                q.put(("aggp", res[(True, True)][2]))
            else:
                q.put(("agp", None))
                q.put(("aggp", None))
            q.put(("gp", g.numpy()))
            q.put(("dm", plane.numpy()))
            q.put(("tb", np.concatenate(parts, axis=1)))
            q.put(("sp", cands))
            q.put(("ts", np.concatenate([p for _, p in sorted(tsr, key=lambda a: a[0])], axis=1)))
            q.put(("tsg", ts_res[True][1]))
            q.put(("tshg", ts_res[("host", True)]))
        # every rank: host_step == __call__ (its own columns)
        np.testing.assert_array_equal(ts_res[("host", False)], ts_res[False][1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sweeps_equal_one_shot(world):
    from oracle import spectra_oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(11))
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    C, N = 16, 1000
    freqs = _band(C)
    dms = np.linspace(0.0, 40.0, 11)
    tab = orc.sweep_table(dms, freqs, DT)
    want = orc.sweep_plane(_data(C, N).astype(np.float64), tab)
    np.testing.assert_array_equal(got["dm"].astype(np.float64), want)
    np.testing.assert_array_equal(got["tb"], want)
    # the pipelined DM-sharded sweep: block of NB spectra, 2 time batches
    want_b = orc.sweep_plane(_data(C, 2400).astype(np.float64), tab)
    np.testing.assert_array_equal(got["ag"].astype(np.float64), want_b)
    np.testing.assert_array_equal(got["agg"].astype(np.float64), want_b)
    np.testing.assert_array_equal(got["gp"].astype(np.float64), want_b)
    if world in (1, 2, 4, 8):
        want_p = orc.sweep_plane(_data(C, 4096).astype(np.float64), tab)
        np.testing.assert_array_equal(got["agp"].astype(np.float64), want_p)
        np.testing.assert_array_equal(got["aggp"].astype(np.float64), want_p)
    np.testing.assert_array_equal(got["ts"].astype(np.float64), want_b)
    np.testing.assert_array_equal(got["tsg"].astype(np.float64), want_b)
    np.testing.assert_array_equal(got["tshg"].astype(np.float64), want_b)
    # sharded search == search of the one-shot plane
    from oracle import search_oracle as so
    xs = _data(C, N)
    xs[:, 300:304] += 60.0
    plane = orc.sweep_plane(xs.astype(np.float64), tab).astype(np.float32)
    c, _ = so.search(plane.astype(np.float64), (1, 2, 4, 8), 5.0, 200)
    sp = got["sp"]
    assert len(sp) == len(c) > 0
    want_k = sorted((dms[d], t, w) for d, t, w, s in c)
    assert sorted(zip(sp["DM"], sp["Sample"], sp["Downfact"])) == want_k


def test_dm_slices_balance():
    s = sharding.dm_slices(10, 3)
    assert s[0][0] == 0 and s[-1][1] == 10
    assert all(a[1] == b[0] for a, b in zip(s, s[1:]))
    # DDplan work weights (1/downsamp): heavier trials spread more thinly
    w = np.r_[np.ones(100), np.full(100, 0.25)]
    sl = sharding.dm_slices(200, 2, w)
    assert sl[0][1] < 100
    assert sharding.dm_slices(3, 8)[-1] == (3, 3)


def test_timeblock_ranges_cover():
    r = sharding.timeblock_ranges(1000, 4, 37)
    assert r[0][0] == 0 and r[-1][1] == 1000
    assert all(b[2] - a[2] == a[1] - a[0] for a, b in zip(r, r[1:]))
    assert all(x[3] - x[1] == 37 for x in r)


@pytest.mark.parametrize("world,nbk,pieces", [(3, 2400, False), (4, 4096, True), (8, 4096, True)])
def test_rehearsal_ranks_stack_to_one_shot(world, nbk, pieces):
    """DMShardedSweep(world=W, rank=r) on one process: every rank's exact
    compute (own slice's corner turn, DM slice at the global width, batch by
    batch) over a shared pre-filled block; the W rank planes stacked are the
    one-shot plane (host logic of bench.py --rehearse; the GPU test runs the
    HIP kernels at the configs[3] geometry)."""
    from oracle import spectra_oracle as orc
    C = 16
    freqs = _band(C)
    dms = np.linspace(0.0, 40.0, 11)
    work = np.r_[np.ones(5), np.full(len(dms) - 5, 0.5)]
    tab = orc.sweep_table(dms, freqs, DT)

    def to_cm(src_tc, dst_cm):
        dst_cm.copy_(src_tc.t())

    def sweep_fn(x, N, piece, x_off, sub, out, n_cols):
        if piece:
            x = x.reshape(N // piece, C, piece).permute(1, 0, 2).reshape(C, N)
        t = orc.sweep_table(sub, freqs, DT)
        xv = x[:, x_off:x_off + n_cols + int(t.max())]
        out.copy_(torch.from_numpy(orc.sweep_plane(xv.numpy().astype(np.float64), t,
                                                   n_out=n_cols).astype(np.float32)))

    block = torch.from_numpy(_data(C, nbk).T.copy())         # time-major [N, C]
    shared, rows = None, []
    for r in range(world):
        ds = sharding.DMShardedSweep(dms, freqs, DT, nbk, dtype=torch.float32, n_batches=2,
                                     work=work, to_cm=to_cm, sweep_fn=sweep_fn, world=world,
                                     rank=r, x_buf=shared)
        assert ds.pieces == pieces and ds.world == world and ds.rank == r
        if shared is None:
            ds.prefill(block)
            shared = ds.x
        ds(sharding.split_block(block, 2, world, r))
        rows.append(ds.plane().numpy())
    want = orc.sweep_plane(_data(C, nbk).astype(np.float64), tab)
    np.testing.assert_array_equal(np.concatenate(rows).astype(np.float64), want)


def test_timeshard_edges():
    e = sharding.timeshard_edges(4179800, 8)
    assert e[0] == 0 and e[-1] == 4179800 and len(e) == 9
    assert all(x % 1024 == 0 for x in e[1:-1])
    w = np.diff(e)
    assert w.max() - w.min() <= 1024 + 4179800 % 1024
    assert sharding.timeshard_edges(100, 4, align=64) == [0, 0, 64, 64, 100]


@pytest.mark.parametrize("world", [1, 3, 8])
def test_timeshard_rehearsal_ranks_concatenate_to_one_shot(world):
    """TimeShardedSweep(world=W, rank=r) on one process: each rank's corner
    turn of its own input spectra (columns + the max-delay overlap) and
    sweep of its columns; the W column blocks concatenate to the one-shot
    plane (host logic of bench.py --rehearse W --mode timeshard)."""
    from oracle import spectra_oracle as orc
    C, N = 16, 3000
    freqs = _band(C)
    dms = np.linspace(0.0, 40.0, 11)
    tab = orc.sweep_table(dms, freqs, DT)

    def to_cm(src_tc, dst_cm):
        dst_cm.copy_(src_tc.t())

    def sweep_fn(x, out, n_cols):
        out.copy_(torch.from_numpy(orc.sweep_plane(x.numpy().astype(np.float64), tab,
                                                   n_out=n_cols).astype(np.float32)))

    block = torch.from_numpy(_data(C, N).T.copy())
    cols = []
    for r in range(world):
        ts = sharding.TimeShardedSweep(dms, freqs, DT, N, dtype=torch.float32, world=world, rank=r,
                                       to_cm=to_cm, sweep_fn=sweep_fn, align=64)
        lo, hi = ts.input_range()
        assert hi - lo == ts.cols + int(tab.max()) and hi <= N
        cols.append(ts(block[lo:hi].contiguous()).numpy().copy())
        # the PCIe-inclusive form (bench.py's end_to_end_pcie leg): the same
        # columns from chunked copies and column ranges
        got = ts.host_step(block[lo:hi].contiguous(), n_batches=3).numpy()
        np.testing.assert_array_equal(got, cols[-1])
    want = orc.sweep_plane(_data(C, N).astype(np.float64), tab)
    np.testing.assert_array_equal(np.concatenate(cols, axis=1).astype(np.float64), want)


def _bench_reduce_worker(rank, world, port, q):
    # bench.py's max-over-ranks timing under the gloo rehearsal backend
    # (PDD_BENCH_BACKEND=gloo: `--gpus N` ranks sharing fewer GPUs)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["PDD_BENCH_BACKEND"] = "gloo"
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "bench_rehearsal", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, bench.max_over_ranks(1.5 * rank + 0.25, None)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_bench_max_over_ranks_gloo():
    """bench.py's per-rank timing reduction (the MAX over ranks of the timed
    region, rank 0 prints the line) over gloo, world size 3."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_reduce_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == {0: 3.25, 1: 3.25, 2: 3.25}
