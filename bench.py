#!/usr/bin/env python
"""Benchmark: the batched brute-force DM sweep.

Default workload = BASELINE.json configs[3], the configuration the metric is
quoted on: ONE 8-bit filterbank block of C = 4096 channels x N = 2^22 samples
swept over D = 4096 DM trials (0-1000 pc/cc, uniform), 64 us sampling,
1250-1550 MHz band, trim=True (plane width N - max delay = 4,179,800),
DM-sharded across the ranks (pypulsar_amd.sharding.DMShardedSweep):
    * the block is resident in HBM in file order (time-major), each rank
      holding its 1/N slice of every time batch (its own H2D share);
    * one step = RCCL all-gathers of the time batches over xGMI, batch k+1's
      gather overlapping batch k's corner turn + sweep, + the sweep of the
      rank's DM slice (balanced by DDplan work fraction, DDplan2b.py:272-273);
      planes stay resident per rank ("strong" scaling: total work fixed);
    * at N = 1 the same path runs without collectives.
Metric: DM-trial samples*channels per second of the whole job
= D * n_out * C per step / step time (max over ranks).
Other workloads: --config config2 (BASELINE configs[1], 1024 x 2^20 x 1024,
float32, time-block mode), northstar (4096 x 2^22 x 2048), stream
(configs[4]), subband (configs[2]), search, ops (incl. configs[0]).

Multi-GPU: `--gpus N` without WORLD_SIZE in the environment starts N ranks
itself (torch.distributed.run on 127.0.0.1, before any GPU call); under
torchrun it uses RANK/LOCAL_RANK/WORLD_SIZE.

Timing: W untimed warm-up steps, then exactly K steps bracketed by a barrier
+ torch.cuda.synchronize(); the max over ranks is reported.  Inside the timed
region every sweep-kernel launch is bracketed by its own HIP event pair on the
stream it runs on (libpdd's event pool, no host syncs); roofline.achieved =
algorithmic adds of those launches / their summed duration.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (MI355X_MICROARCH.md §Chip-level parameters, §LDS)
PEAK_HBM_GBS = 8000.0
CLK_GHZ = 2.4
N_CU = 256
# LDS ds_read_b128: 256 B/clk/CU (MI355X_MICROARCH.md §LDS table)
LDS_B_PER_CLK = 256
# VALU: 4 SIMD-32 per CU, a wave64 instruction over 2 cycles (MI355X_MICROARCH.md
# :53-54) = 128 lane-ops/clk/CU = 78.6 T lane-ops/s chip-wide
VALU_LANE_OPS_T = N_CU * 4 * 32 * CLK_GHZ / 1e3
PEAK_ADD_T = VALU_LANE_OPS_T * 2   # v_pk_add_f32 / v_add_u32 on packed u16: 2 adds per lane-op

CONFIGS = {
    # BASELINE.json configs[3] (the metric's configuration): DM-sharded node sweep
    "config3": dict(C=4096, N=1 << 22, D=4096, dm_lo=0.0, dm_hi=1000.0, dtype="u8",
                    mode="auto", cpu=(4096, 1 << 17, 12), baseline_index=3),
    # BASELINE.json configs[1]: single-GPU brute-force sweep, float32
    "config2": dict(C=1024, N=1 << 20, D=1024, dm_lo=0.0, dm_hi=1000.0, dtype="f32",
                    mode="timeblock", cpu=(1024, 1 << 20, 3), baseline_index=1),
    # north-star single-GPU target (4096 ch x 2048 DM x 2^22)
    "northstar": dict(C=4096, N=1 << 22, D=2048, dm_lo=0.0, dm_hi=1000.0, dtype="u8",
                      mode="auto", cpu=(4096, 1 << 17, 12), baseline_index=None),
    "small": dict(C=256, N=1 << 18, D=256, dm_lo=0.0, dm_hi=500.0, dtype="f32",
                  mode="timeblock", cpu=(256, 1 << 18, 8), baseline_index=None),
    # BASELINE.json configs[4]: streaming u8 blocks, zero-DM + ds 2 + 2048 DMs
    "stream": dict(C=4096, N=1 << 18, D=2048, dm_lo=0.0, dm_hi=1000.0, ds=2),
    # BASELINE.json configs[2]: two-stage subband sweep over a DDplan2b grid
    "subband": dict(C=4096, N=1 << 20, nsub=64, dm_lo=0.0, dm_hi=1000.0, res=0.5),
    # single-pulse search over the config2 plane
    "search": dict(C=1024, N=1 << 20, D=1024, dm_lo=0.0, dm_hi=1000.0),
    # HBM-bound single-DM kernels at a large block,
    # plus BASELINE.json configs[0] (waterfaller dedisperse, 1024 x 2^16, DM 100)
    "ops": dict(C=4096, N=1 << 18, wf_C=1024, wf_N=1 << 16, wf_dm=100.0),
}


def _factor_arg(args):
    """DMSweep(factor=...) of the --factor option."""
    return {"auto": True, "off": False, "2": 2, "4": 4, "force2": "force2",
            "force4": "force4"}[args.factor]


def log(*a):
    print("[bench %s]" % time.strftime("%H:%M:%S"), *a, file=sys.stderr, flush=True)


def band(C, lo=1250.0, hi=1550.0):
    foff = -(hi - lo) / C
    return (hi + foff / 2.0) + foff * np.arange(C)


def synth_block(C, N, seed, dtype, device, rows_per_chunk=1 << 26):
    """uint8 clip(round(N(128, 16))) filterbank block [C, N], generated on the
    device in row chunks (bounded float32 temporaries)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty((C, N), dtype=torch.uint8 if dtype == "u8" else torch.float32,
                      device=device)
    step = max(1, rows_per_chunk // max(N, 1))
    for r in range(0, C, step):
        x = torch.empty((min(step, C - r), N), dtype=torch.float32, device=device)
        x.normal_(128.0, 16.0, generator=g)
        x = x.round_().clamp_(0, 255)
        out[r:r + x.shape[0]] = x.to(out.dtype)
        del x
    return out


def cpu_baseline(C, n, dms, ntrials, dt, full_N):
    """Oracle (NumPy restatement of Spectra.dedisperse + channel sum, C-order,
    one core) on a BOUNDED sample of the workload: ``ntrials`` DM trials of
    the grid (spread over it) on a C x n block (n <= the workload's N)."""
    from oracle import spectra_oracle as orc
    freqs = band(C)
    rng = np.random.default_rng(0)
    x = np.clip(np.round(rng.normal(128, 16, (C, n))), 0, 255).astype(np.float64)
    pick = dms[np.linspace(0, len(dms) - 1, ntrials).astype(int)]
    work = 0
    t0 = time.perf_counter()
    for dm in pick:
        d, _ = orc.dedisperse(x, freqs, dt, dm, padval=0, trim=True)
        s = orc.channel_sum(d)
        work += s.shape[0] * C
        del d, s
    el = time.perf_counter() - t0
    res = dict(value=work / el, unit="samples*channels*DM/s", cores=1, kind="port",
               sample="%d DM trials of the grid (dedisperse(trim=True)+channel sum), "
                      "%d ch x %d samples (workload: %d), float64 NumPy C-order, 1 thread, "
                      "%.1f s" % (ntrials, C, n, full_N, el))
    res["cpu_model"] = _cpu_model()
    res["nproc"] = os.cpu_count()
    res["f_order_1core"] = _cpu_forder(x, freqs, dt, pick[-1], orc)
    res["all_cores"] = _cpu_pool(x, freqs, dt, dms, orc)
    return res


def _pinned_h2d_GBs(h, dev, reps=5):
    """Pinned host -> device rate of ``h`` copied alone (best of ``reps``)."""
    d = torch.empty(h.shape, dtype=h.dtype, device=dev)
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    del d
    return h.numel() * h.element_size() / best / 1e9


def stream_cpu_baseline(C, ds, dms, dt, nb_gpu, D, mode, n_raw=1 << 17, ntrials=12):
    """The stream's per-block work on the host: the oracle's
    zero-DM (the reference's uint8 result, bin/zero_dm_filter.py:30-39, per
    spectrum) + downsample (formats/spectra.py:329-351) of an ``n_raw``-
    spectrum 8-bit slice, then ``ntrials`` DM trials of dedisperse(trim) +
    channel sum (spectra.py:229-260, waterfaller.py:140), one core, C-order.
    ``value`` extrapolates the timed sample to the GPU's per-block work: one
    prologue + D trials per block of units D x columns x C."""
    from oracle import spectra_oracle as orc
    freqs = band(C)
    rng = np.random.default_rng(1)
    x = np.clip(np.round(rng.normal(128, 16, (n_raw, C))), 0, 255).astype(np.uint8)
    zmode = {"wrap": "wrap", "int": "int"}.get(mode, "none")
    t0 = time.perf_counter()
    if mode == "float":
        z = orc.zdm_downsample(x, ds, zero_dm=True)
    else:
        z = orc.zdm_int_downsample(x, ds, mode=zmode).astype(np.float64)
    z = np.ascontiguousarray(z)  # [C, n] channel rows, C-order (as Spectra.data)
    t_pro = time.perf_counter() - t0
    pick = dms[np.linspace(0, len(dms) - 1, ntrials).astype(int)]
    cols, t0 = [], time.perf_counter()
    for dm in pick:
        d, _ = orc.dedisperse(z, freqs, dt * ds, dm, padval=0, trim=True)
        cols.append(orc.channel_sum(d).shape[0])
        del d
    t_tr = (time.perf_counter() - t0) / ntrials
    n_cols = float(np.mean(cols))
    value = D * n_cols * C / (t_pro + D * t_tr)
    return dict(value=value, unit="samples*channels*DM/s (downsampled samples)", cores=1,
                kind="port", cpu_model=_cpu_model(), nproc=os.cpu_count(),
                prologue_s=t_pro, s_per_trial=t_tr,
                sample="zero-DM (%s) + downsample %d of %d x %d u8 spectra (%.2f s), then %d DM "
                       "trials of the grid (dedisperse(trim)+channel sum) on the %d x %d "
                       "result (%.2f s each), float64 NumPy, 1 thread; value = one prologue "
                       "+ %d trials per block" % (mode, ds, n_raw, C, t_pro, ntrials, C,
                                                  z.shape[1], t_tr, D))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cpu_forder(x, freqs, dt, dm, orc, n=1 << 16):
    """One trial on the F-order layout get_spectra produces (filterbank.py:
    155-157 reshape + .T), where the reference's per-channel rotate walks
    strided rows: first ``n`` samples only, per unit."""
    n = min(n, x.shape[1])
    xf = np.asfortranarray(x[:, :n])
    t0 = time.perf_counter()
    d, _ = orc.dedisperse(xf, freqs, dt, dm, padval=0, trim=True)
    s = orc.channel_sum(d)
    el = time.perf_counter() - t0
    return dict(value=s.shape[0] * x.shape[0] / el, cores=1,
                sample="1 DM trial (DM %.1f) on F-order %d ch x %d samples, %.1f s"
                       % (dm, x.shape[0], n, el))


def lease_cpus():
    """Host CPUs this process may use: the affinity mask, capped by the
    lease's thread budget where one is set (the GPU box exports
    OMP_NUM_THREADS = its CPU share; nproc there shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def _cpu_pool(x, freqs, dt, dms, orc, workers=None, ntrials=None, cblk=64):
    """DM-parallel variant on every core of the lease: one
    fresh interpreter per core (``python -m oracle.cpu_pool``: NumPy + the
    oracle only, so no GPU file descriptor is inherited and the card's
    process limit does not cap the pool), each mapping the same block from
    a .npy in /dev/shm and running its share of (DM trial, channel block)
    tasks of the reference algorithm; timed from one "go" to the last
    result."""
    import shutil
    import tempfile
    workers = workers or lease_cpus()
    ntrials = ntrials or 2 * workers
    C, N = x.shape
    pick = dms[np.linspace(0, len(dms) - 1, ntrials).astype(int)]
    tasks = []
    for dm in pick:
        bins = orc.dedisperse_bins(dm, 0.0, freqs, dt)
        n_keep = N - max(0, int(bins.max()))
        tasks += [[c, min(C, c + cblk), float(dm), n_keep] for c in range(0, C, cblk)]
    workers = min(workers, len(tasks))
    tmpdir = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    procs = []
    try:
        path = os.path.join(tmpdir, "x.npy")
        np.save(path, np.ascontiguousarray(x))
        env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
        for w in range(workers):
            p = subprocess.Popen([sys.executable, "-m", "oracle.cpu_pool"], cwd=ROOT, env=env,
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
            p.stdin.write(json.dumps({"x": path, "freqs": list(map(float, freqs)), "dt": dt,
                                      "tasks": tasks[w::workers]}) + "\n")
            p.stdin.flush()
            procs.append(p)
        for p in procs:
            assert p.stdout.readline().strip() == "ready", "cpu_pool worker failed"
        t0 = time.perf_counter()
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.flush()
        res = [json.loads(p.stdout.readline()) for p in procs]
        el = time.perf_counter() - t0
        for p in procs:
            p.wait(timeout=60)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        shutil.rmtree(tmpdir, ignore_errors=True)
    work = sum(r["work"] for r in res)
    return dict(value=work / el, cores=workers, lease_cpus=lease_cpus(),
                sample="%d DM trials on the same block split into %d-channel blocks over %d "
                       "single-threaded worker processes (one per lease CPU), float64 NumPy "
                       "C-order, %.1f s" % (ntrials, cblk, workers, el))


def load_pmc(path, key, plan=None, ctx=None):
    """profiles/pmc_sweep.json[key] if it was measured on THIS binary and run:
    the entry's source digest (scripts/collect_profiles.py) must equal the
    digest compiled into the LOADED libpdd.so, its sweep plan the running
    plan and its run context (mode, world size, launches per step = columns
    per launch) this run's; anything else is refused (None)."""
    try:
        with open(path) as f:
            e = json.load(f).get(key)
        if not isinstance(e, dict):
            return None
        from pypulsar_amd._lib import loaded_digest
        if e.get("src_digest") != loaded_digest():
            return None
    except Exception:
        return None
    if plan is not None and e.get("plan") is not None and e.get("plan") != plan:
        return None
    if ctx is not None and e.get("ctx") != ctx:
        return None
    return e


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# PDD_BENCH_BACKEND=gloo: rehearse `--gpus N` with N ranks on the GPUs this
# box has (one here), barriers and the max-over-ranks timing over gloo; the
# driver's multi-GPU runs use RCCL ("nccl"), one rank per GPU
_BACKEND = os.environ.get("PDD_BENCH_BACKEND", "nccl")


def max_over_ranks(v, dev):
    """The maximum of a per-rank float over all ranks (RCCL: on the device)."""
    t = torch.tensor([float(v)], dtype=torch.float64, device=dev if _BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _maybe_spawn(args):
    """`--gpus N` outside torchrun: start N ranks (one per GPU) with
    torch.distributed.run before this process touches the GPU, and exit with
    their status."""
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="config3", choices=sorted(CONFIGS))
    ap.add_argument("--block", type=int, default=None, help="stream: spectra per block")
    ap.add_argument("--dtype", default=None, choices=["f32", "u8"])
    ap.add_argument("--mode", default=None, choices=["timeblock", "dmshard", "timeshard", "auto"],
                    help="config3/northstar: dmshard (DM slices, RCCL all-gathers), timeshard "
                         "(column ranges of the same block, no collective) or auto (the "
                         "default: dmshard at N = 1, timeshard at N > 1 -- bench.py "
                         "--rehearse 8 measures both, DESIGN.md §5)")
    ap.add_argument("--batches", type=int, default=None,
                    help="dmshard: time batches per step (default 1 on one GPU, 4 otherwise)")
    ap.add_argument("--gather", action="store_true",
                    help="dmshard: also gather every batch's plane rows to rank 0 (p2p)")
    ap.add_argument("--zdm", default="auto", choices=["auto", "int", "wrap", "float", "none"],
                    help="stream: zero-DM mode (auto = 'wrap', the reference's uint8 result of "
                         "zero_dm_filter.py:30-39, on the exact 16-bit path)")
    ap.add_argument("--cpu-trials", type=int, default=None)
    ap.add_argument("--factor", default="auto", choices=["auto", "off", "2", "4", "force2", "force4"],
                    help="8-bit sweeps: exact factorisation over channel groups (auto = the "
                         "planner's cost model picks 4, 2 or none; off = channel by channel; "
                         "2 / 4 = that group size where it pays; force2 / force4 = that size "
                         "wherever it fits)")
    ap.add_argument("--no-skew", action="store_true",
                    help="factorised sweeps: plane-aligned tiles instead of delay-aligned ones "
                         "(the A/B of DESIGN.md §3.2; the plane is identical)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="dmshard / timeshard: skip the PCIe-inclusive (pinned host -> H2D -> "
                         "step) leg")
    ap.add_argument("--e2e", action="store_true",
                    help="also time one PCIe-inclusive step: pinned host block -> H2D -> "
                         "sweep -> D2H of the plane into pinned host memory")
    ap.add_argument("--search", action="store_true",
                    help="stream: also boxcar-search every block (StreamingSearch)")
    ap.add_argument("--rehearse", type=int, default=0, metavar="W",
                    help="dmshard: run every rank of a W-GPU step on this one GPU (its own "
                         "slice's corner turn + its DM slice) and report per-rank times and the "
                         "predicted compute efficiency")
    args = ap.parse_args()
    _maybe_spawn(args)
    if args.no_skew:
        from pypulsar_amd import sweep as _sweep_mod
        _sweep_mod.TEST_SWITCHES["no_skew"] = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if _BACKEND == "gloo":
        # rehearsal of the N-rank code path on fewer GPUs (gloo: CPU
        # barriers/reductions; the ranks share the visible GPUs)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and _BACKEND == "gloo":
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import __graft_entry__ as g
    if rank == 0:
        g.build()
    if world > 1:
        dist.barrier()
    g.build()

    cfg = CONFIGS[args.config]
    if args.config in ("stream", "subband", "search", "ops"):
        args.steps = 10 if args.steps is None else args.steps
        args.warmup = 3 if args.warmup is None else args.warmup
    if args.config == "stream":
        return stream_bench(args, cfg, rank, world, dev)
    if args.config == "subband":
        return subband_bench(args, cfg, rank, world, dev)
    if args.config == "search":
        return search_bench(args, cfg, rank, world, dev)
    if args.config == "ops":
        return ops_bench(args, cfg, rank, world, dev)
    if args.rehearse and (args.mode or "dmshard") == "timeshard":
        return rehearse_timeshard(args, cfg, dev)
    if args.rehearse:
        return rehearse_bench(args, cfg, dev)
    return sweep_bench(args, cfg, rank, world, dev)


def sweep_bench(args, cfg, rank, world, dev):
    from pypulsar_amd.sweep import DMSweep
    from pypulsar_amd.sharding import DMShardedSweep, TimeShardedSweep, trial_work
    big = cfg["C"] * cfg["N"] >= (1 << 34)
    steps = args.steps if args.steps is not None else (5 if big else 10)
    warmup = args.warmup if args.warmup is not None else (1 if big else 3)
    C, N, D = cfg["C"], cfg["N"], cfg["D"]
    dtype = args.dtype or cfg["dtype"]
    mode = args.mode or cfg["mode"]
    if mode == "auto":
        mode = "dmshard" if world == 1 else "timeshard"
    dt = 64e-6
    freqs = band(C)
    dms_all = np.linspace(cfg["dm_lo"], cfg["dm_hi"], D)
    tdt = torch.uint8 if dtype == "u8" else torch.float32
    nb = None
    if mode == "dmshard":
        # 4 time batches at every N: the all-gather of batch k+1 (N > 1) or
        # the H2D of batch k+1 (the PCIe-inclusive leg) overlaps batch k's sweep
        nb = args.batches or 4
        # uniform grid = one DDstep at downsamp 1: every trial weighs 1/1
        # (DDplan2b.py:272-273); DMShardedSweep balances the slices by it
        ds = DMShardedSweep(dms_all, freqs, dt, N, dtype=tdt, n_batches=nb,
                            work=trial_work(dms_all, 1), gather=args.gather, device=dev,
                            factor=_factor_arg(args))
        log("rank %d: DM slice [%d, %d) of %d, %d batch(es)" % (rank, ds.lo, ds.hi, D, nb))
        # this rank's H2D share of every time batch, [nb, N/(nb*world), C],
        # in file (time-major) order
        n_r = N // (nb * world)
        part = synth_block(nb * n_r, C, 1000 + rank, dtype, dev).view(nb, n_r, C)
        sw, rows, n_out = ds.sw, ds.rows, ds.n_out
        cols_rank, n_in_rank = n_out, N

        def step():
            return ds(part)
    elif mode == "timeshard":
        # column ranges of the same block: rank r holds its own input spectra
        # (columns + the max-delay overlap, time-major, its own H2D), no
        # collective (pypulsar_amd.sharding.TimeShardedSweep)
        ts = TimeShardedSweep(dms_all, freqs, dt, N, dtype=tdt, gather=args.gather, device=dev,
                              factor=_factor_arg(args))
        log("rank %d: plane columns [%d, %d) of %d, input spectra [%d, %d)"
            % (rank, ts.a, ts.b, ts.n_out, ts.in_lo, ts.in_hi))
        part = synth_block(ts.n_in, C, 1000 + rank, dtype, dev)   # [n_in, C] file order
        sw, rows, n_out = ts.sw, D, ts.n_out
        cols_rank, n_in_rank = ts.cols, ts.n_in

        def step():
            return ts(part)
    else:
        x = synth_block(C, N, 1000 + rank, dtype, dev)
        sw = DMSweep(dms_all, freqs, dt, dtype=dtype, factor=_factor_arg(args))
        rows, n_out = D, sw.n_out(N)
        cols_rank, n_in_rank = n_out, N
        plane = torch.empty((D, n_out), dtype=torch.float32, device=dev)

        def step():
            return sw(x, out=plane)
    log("rank %d: block synthesised; warm-up x%d" % (rank, warmup))
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if sw is not None:
        sw.set_timing(True)  # event pair per sweep launch, no host syncs
    log("rank %d: timing %d steps" % (rank, steps))
    t0 = time.perf_counter()
    for i in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms, launches = sw.timing_read() if sw is not None else (0.0, 0)
    if sw is not None:
        sw.set_timing(False)
    e2e = None
    if mode == "dmshard" and not args.no_e2e:
        # PCIe-inclusive: this rank's slices of the block in
        # pinned host memory -> H2D -> the step; planes stay resident (the
        # consumer is the on-device search), so no plane D2H
        hpart = torch.empty(part.shape, dtype=part.dtype, pin_memory=True)
        hpart.copy_(part)
        ms, h2d = [], []
        copy_stream = torch.cuda.Stream(device=dev)
        landed = [torch.cuda.Event() for _ in range(nb)]
        cur = torch.cuda.current_stream(dev)
        for _ in range(3):
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
            # H2D alone (timed once per repetition for the rate)
            part.copy_(hpart, non_blocking=True)
            torch.cuda.synchronize()
            h2d.append((time.perf_counter() - t1) * 1e3)
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
            if world == 1:
                # batch k+1's H2D (copy stream) overlaps batch k's corner turn + sweep
                copy_stream.wait_stream(cur)
                with torch.cuda.stream(copy_stream):
                    for k in range(nb):
                        part[k].copy_(hpart[k], non_blocking=True)
                        landed[k].record(copy_stream)
                for k in range(nb):
                    cur.wait_event(landed[k])
                    ds.exchange_batch(part, k)
                    ds.sweep_batch(k)
            else:
                part.copy_(hpart, non_blocking=True)
                step()
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t1) * 1e3)
        del hpart
        best = min(ms)
        if world > 1:
            best = max_over_ranks(best, dev)
        nbytes = part.numel() * part.element_size()
        e2e = {"ms_per_step": best, "value": D * n_out * C / (best * 1e-3),
               "h2d_ms": min(h2d), "h2d_GBs": nbytes / (min(h2d) * 1e-3) / 1e9,
               "bytes_h2d_per_rank": nbytes, "bytes_d2h": 0,
               "note": "best of 3 (max over ranks): pinned host slices -> H2D (this rank's 1/N "
                       "of every time batch) -> the step; planes stay resident per rank (the "
                       "consumer is the on-device search), so nothing returns over PCIe; at "
                       "N = 1 the H2D of time batch k+1 runs on a copy stream under batch k's "
                       "sweep, at N > 1 the whole slice is copied before the step"}
    if mode == "timeshard" and not args.no_e2e:
        # PCIe-inclusive: this rank's input spectra (its
        # columns + the max-delay overlap) in pinned host memory -> H2D in 4
        # chunks on a copy stream, the columns swept in 4 ranges as their
        # chunks land (TimeShardedSweep.host_step); planes stay resident
        hpart = torch.empty(part.shape, dtype=part.dtype, pin_memory=True)
        hpart.copy_(part)
        cs = torch.cuda.Stream(device=dev)
        ms, h2d = [], []
        for _ in range(3):
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
            part.copy_(hpart, non_blocking=True)
            torch.cuda.synchronize()
            h2d.append((time.perf_counter() - t1) * 1e3)
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
            ts.host_step(hpart, n_batches=4, copy_stream=cs)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t1) * 1e3)
        del hpart
        best = min(ms)
        h2d_best = min(h2d)
        if world > 1:
            best = max_over_ranks(best, dev)
            h2d_best = max_over_ranks(h2d_best, dev)
        nbytes = part.numel() * part.element_size()
        e2e = {"ms_per_step": best, "value": D * n_out * C / (best * 1e-3),
               "h2d_ms": h2d_best, "h2d_GBs": nbytes / (h2d_best * 1e-3) / 1e9,
               "bytes_h2d_per_rank": nbytes, "bytes_d2h": 0,
               "note": "best of 3 (max over ranks): each rank's input spectra (plane columns + "
                       "the max-delay overlap) in pinned host memory -> H2D in 4 chunks on a "
                       "copy stream, the columns swept in 4 ranges as their chunks land "
                       "(chunk k+1's copy under range k's corner turn + sweep; chunk 0's "
                       "exposed); planes stay resident per rank, nothing returns over PCIe"}
    if args.e2e and mode == "timeblock":
        # PCIe-inclusive: the boundary handed host buffers
        hx = torch.empty(x.shape, dtype=x.dtype, pin_memory=True)
        hx.copy_(x)
        hp = torch.empty(plane.shape, dtype=plane.dtype, pin_memory=True)
        xd = torch.empty_like(x)
        ms = []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            xd.copy_(hx, non_blocking=True)
            sw(xd, out=plane)
            hp.copy_(plane, non_blocking=True)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t1) * 1e3)
        e2e = {"ms_per_step": min(ms), "value": D * n_out * C / (min(ms) * 1e-3),
               "bytes_h2d": x.numel() * x.element_size(), "bytes_d2h": plane.numel() * 4,
               "note": "best of 3; value = samples*channels*DM/s including the transfers"}
        del hx, hp, xd
    rccl_world = dist.get_world_size() if world > 1 else 1
    if world > 1:
        el = max_over_ranks(el, dev)
    adds_rank_step = rows * cols_rank * C        # one add per samp*ch*DM on this rank
    units_all = D * n_out * C * (world if mode == "timeblock" else 1)
    value = units_all * steps / el
    s_in = 1 if dtype == "u8" else 4
    # exact factorised 8-bit sweep: the kernel adds one
    # pattern sample per (trial, group of fx channels), so its own adds are
    # C / fx per samp*DM; the algorithmic rate is reported beside them
    fx_g, fx_pat = sw.factor_info(1 if dtype == "u8" else 0) if sw is not None else (0, 0)
    kern_adds_step = rows * cols_rank * (C // fx_g) if fx_g else adds_rank_step
    achieved = kern_adds_step * steps / (kern_ms * 1e-3) / 1e12 if kern_ms > 0 else None
    effective = adds_rank_step * steps / (kern_ms * 1e-3) / 1e12 if kern_ms > 0 else None
    # LDS roof (the binding one): ds_read_b128 at 256 B/clk/CU
    # feeds 4 f32 samples (f32 quarters) or 8 u16 samples (u16 eighths) per 16 B
    lds_roof = N_CU * CLK_GHZ * 1e9 * LDS_B_PER_CLK / 16 * (8 if dtype == "u8" else 4) / 1e12
    # VALU roof: u16 eighths add two channels of two packed samples per
    # v_add3_u32 lane-op (4 adds); f32 quarters two samples per v_pk_add_f32
    valu_adds = 4 if dtype == "u8" else 2
    valu_roof = VALU_LANE_OPS_T * valu_adds
    uniq_bytes = C * n_in_rank * s_in + rows * cols_rank * 4
    k_s = kern_ms * 1e-3 / steps if kern_ms > 0 else None
    # keys of profiles/pmc_sweep.json (scripts/collect_profiles.py): the
    # default configs[3] line (factorised), its channel-kernel line, ...
    pmc_key = "%s_%s" % (args.config, dtype)
    if args.config == "config3" and not fx_g:
        pmc_key = "config3_channel"
    elif args.config == "northstar":
        pmc_key = "northstar"
    plan = sw.info(1 if dtype == "u8" else 0) if sw is not None else None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_sweep.json")
    lps = launches / steps if launches else None
    ctx = {"mode": mode, "world": world, "launches_per_step": lps}
    pmc = load_pmc(pmc_path, pmc_key, plan, ctx)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    pmc1 = load_pmc(pmc_path, pmc_key + "_stage1", plan, ctx) if fx_g else None
    # per step: the sweep kernel's (and stage 1's) counter bytes per launch x
    # launches per step, against the algorithmic bytes (input once + plane once)
    traffic_step = None
    if traffic and lps:
        traffic_step = (traffic + (pmc1.get("hbm_bytes_per_launch") if pmc1 else 0.0)) * lps

    if rank == 0:
        line = {
            "metric": "DM-trial samples*channels/sec (node) + % HBM roofline",
            "value": value,
            "unit": "samples*channels*DM/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": el / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if mode == "timeblock" else "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (uint8 clip(round(N(128,16))) filterbank%s, generated on device)"
                    % ("" if dtype == "u8" else " as float32"),
            "config": {"workload": "%s: DM sweep %d ch x 2^%d samples x %d DM "
                                   "(%g-%g pc/cc), 64 us, 1250-1550 MHz, trim=True, every plane "
                                   "row = the brute-force per-trial channel sum%s"
                                   % ("BASELINE configs[%d]" % cfg["baseline_index"]
                                      if cfg["baseline_index"] is not None else args.config,
                                      C, int(np.log2(N)), D, cfg["dm_lo"], cfg["dm_hi"],
                                      ", DM-sharded (RCCL all-gather of per-rank time-batch "
                                      "slices, %d batch(es), planes %s)"
                                      % (nb, "gathered to rank 0" if args.gather else
                                         "resident per rank") if mode == "dmshard" else
                                      (", time-sharded (each rank a contiguous range of plane "
                                       "columns from its own input spectra + the max-delay "
                                       "overlap, no collective, planes %s)"
                                       % ("gathered to rank 0" if args.gather else
                                          "resident per rank") if mode == "timeshard" else
                                       ", every rank its own block")),
                       "config_name": args.config, "channels": C, "samples": N, "dm_trials": D,
                       "n_out": n_out, "mode": mode,
                       "parallelism": "%s%d" % ({"timeblock": "tb", "timeshard": "ts"}
                                                .get(mode, "dm"), world),
                       "rccl_world_size": rccl_world if _BACKEND == "nccl" else 0,
                       "dist_backend": (_BACKEND if world > 1 else None), "plan": plan,
                       "method": (("exact factorisation over groups of %d channels (%d pattern "
                                   "series; plane bit-identical to the channel-by-channel sum)"
                                   if dtype == "u8" else
                                   "factorisation over groups of %d channels (%d float32 pattern "
                                   "series; the channel sum regrouped: within the float32 bar, "
                                   "exact for integer-valued data)")
                                  % (fx_g, fx_pat) if fx_g else "channel by channel")},
            "roofline": {"bound": "lds", "achieved": achieved, "peak": lds_roof,
                         "unit": "T adds/s", "frac": achieved / lds_roof if achieved else None,
                         "traffic": traffic,
                         "traffic_source": ("profiles/pmc_sweep.json[%s]: separate rocprofv3 "
                                            "--pmc FETCH_SIZE / WRITE_SIZE passes of this "
                                            "command, kernel %s, commit %s, source digest %s "
                                            "(= this build)" % (pmc_key, pmc.get("kernel"),
                                                                pmc.get("commit"),
                                                                pmc.get("src_digest")))
                         if traffic else "no profiles/pmc_sweep.json[%s] entry of this build, "
                                         "plan and run context (%s): traffic not reported"
                                         % (pmc_key, json.dumps(ctx, sort_keys=True)),
                         "traffic_stage1": pmc1.get("hbm_bytes_per_launch") if pmc1 else None,
                         "traffic_unit": "HBM-side bytes per launch (traffic: this kernel; "
                                         "traffic_stage1: the factorised stage 1)",
                         "traffic_per_step": traffic_step,
                         "algorithmic_bytes_per_step": uniq_bytes,
                         "traffic_ratio": traffic_step / uniq_bytes if traffic_step else None,
                         "kernel": ("pdd::k_sweep_il (factorised stage 2)" if fx_g
                                    else "pdd::k_sweep_il"), "kernel_ms_per_launch":
                             kern_ms / launches if launches else None,
                         "launches_per_step": launches / steps if launches else None,
                         "kernel_s_per_step": k_s,
                         "adds_per_step_rank0": kern_adds_step,
                         "units_per_step_rank0": adds_rank_step,
                         "effective_units_T_per_s": effective,
                         "note": ("factorised stage 2: one add per samp*DM*(group of %d "
                                  "channels), each reading its pattern sample from the LDS image "
                                  "(ds_read_b128: %d samples per 16 B at 256 B/clk/CU = the peak, "
                                  "in adds/s); the tile is bound by staging the pattern windows "
                                  "(LDS-DMA), so the LDS-read fraction is low by construction; "
                                  "effective_units_T_per_s = samp*ch*DM per second of this "
                                  "kernel (DESIGN.md §3-4)" % (fx_g, 8 if dtype == "u8" else 4))
                         if fx_g else
                                 ("one add per samp*ch*DM, no MFMA-shaped work; every add reads "
                                  "its sample from the LDS image (ds_read_b128: %d samples per 16 B "
                                  "at 256 B/clk/CU = the peak, in adds/s), which binds; the VALU "
                                  "issue rate (SIMD-32, MI355X_MICROARCH.md:53-54) is beside it "
                                  "(DESIGN.md §3-4)" % (8 if dtype == "u8" else 4)),
                         "lds_bytes_per_add": 2 if dtype == "u8" else 4,
                         "valu": {"peak": valu_roof, "unit": "T adds/s",
                                  "instr": ("v_add3_u32 over a channel pair of packed u16 samples "
                                            "(4 adds per lane-op)" if dtype == "u8" else
                                            "v_pk_add_f32 (2 adds per lane-op)"),
                                  "lane_ops_T": VALU_LANE_OPS_T,
                                  "frac": achieved / valu_roof if achieved else None}},
            "roofline_hbm": {"bound": "hbm", "achieved": uniq_bytes / k_s / 1e9 if k_s else None,
                             "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": uniq_bytes / k_s / 1e9 / PEAK_HBM_GBS if k_s else None,
                             "bytes_per_step": uniq_bytes,
                             "note": "unique bytes (input once + plane once) over the sweep "
                                     "kernel time: capped at a few % for a sweep (SURVEY.md "
                                     "§8(d))"},
            "cpu_baseline": None,
        }
        if e2e is not None:
            line["end_to_end_pcie"] = e2e
        if world == 1 and not args.no_cpu_baseline:
            del step
            if mode in ("dmshard", "timeshard"):
                del part
            else:
                del x
            torch.cuda.empty_cache()
            cC, cn, ct = cfg["cpu"]
            log("cpu baseline: %d ch x %d samples, %d trials" % (cC, cn, ct))
            line["cpu_baseline"] = cpu_baseline(cC, cn, dms_all, args.cpu_trials or ct, dt, N)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def rehearse_bench(args, cfg, dev):
    """The W-rank DM-sharded step (BASELINE configs[3] by default) rehearsed on
    ONE GPU: first the whole grid as one rank (the N=1 step), then rank r =
    0..W-1 exactly as it runs in a W-GPU job (DMShardedSweep(world=W,
    rank=r): its own slice of each of the 4 time batches corner-turned into
    the pieces block, its DDplan-work-balanced DM slice -- DDplan2b.py:272-273
    -- swept at the global width), the all-gathers replaced by a block that
    already holds every rank's slices.  Reports per-rank step and sweep-kernel
    times, trial-block rounding and the predicted compute-side efficiency
    t(1 GPU) / (W * max_r t_r); the exchange (all-gathers over xGMI) is not
    part of it and is modelled in DESIGN.md §5."""
    from pypulsar_amd.sharding import DMShardedSweep, split_block, trial_work
    W = args.rehearse
    C, N, D = cfg["C"], cfg["N"], cfg["D"]
    dtype = args.dtype or cfg["dtype"]
    tdt = torch.uint8 if dtype == "u8" else torch.float32
    dt = 64e-6
    freqs = band(C)
    dms = np.linspace(cfg["dm_lo"], cfg["dm_hi"], D)
    nb = args.batches or 4
    steps = args.steps if args.steps is not None else 3
    warmup = args.warmup if args.warmup is not None else 1
    block = synth_block(N, C, 1000, dtype, dev)            # time-major [N, C], file order

    def timed(ds, part):
        for _ in range(warmup):
            ds(part)
        torch.cuda.synchronize()
        ds.sw.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            ds(part)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        kms, launches = ds.sw.timing_read()
        ds.sw.set_timing(False)
        return el, kms / steps, launches // steps

    # the N = 1 step (whole grid, one rank, nb = 1 as in the default bench line)
    ds1 = DMShardedSweep(dms, freqs, dt, N, dtype=tdt, n_batches=1, work=trial_work(dms, 1),
                         device=dev, factor=_factor_arg(args))
    t1, k1, l1 = timed(ds1, block.view(1, N, C))
    db = ds1.sw.info(1 if dtype == "u8" else 0)["dms_per_block"]
    fx1 = ds1.sw.factor_info(1 if dtype == "u8" else 0)
    ds1.close()
    del ds1
    torch.cuda.empty_cache()
    log("rehearse: 1 GPU step %.1f ms (sweep %.1f ms, %d launches)" % (t1, k1, l1))
    ranks, shared = [], None
    for r in range(W):
        ds = DMShardedSweep(dms, freqs, dt, N, dtype=tdt, n_batches=nb, work=trial_work(dms, 1),
                            device=dev, world=W, rank=r, x_buf=shared, factor=_factor_arg(args))
        if shared is None:
            ds.prefill(block)
            shared = ds.x
        part = split_block(block, nb, W, r)
        t, k, l = timed(ds, part)
        blocks = -(-ds.rows // db)
        code = 1 if dtype == "u8" else 0
        g, npat = ds.sw.factor_info(code)
        # stage 1's pattern image of the rank's slice (bytes written per batch)
        pbytes = ds.sw.pattern_bytes(max(ds.col_edges[1] - ds.col_edges[0], 1), code) if g else 0
        ranks.append({"rank": r, "dms": [ds.lo, ds.hi], "rows": ds.rows, "step_ms": t,
                      "sweep_kernel_ms": k, "launches": l, "trial_blocks": blocks,
                      "trial_block_fill": ds.rows / (blocks * db),
                      "outside_stage2_ms": t - k, "fx": [g, npat],
                      "pattern_bytes_per_batch": pbytes})
        log("rehearse: rank %d/%d DMs [%d, %d) step %.1f ms (sweep %.1f ms)"
            % (r, W, ds.lo, ds.hi, t, k))
        ds.close()
        del ds, part
        torch.cuda.empty_cache()
    tmax = max(x["step_ms"] for x in ranks)
    line = {
        "metric": "rehearsal of the %d-GPU DM-sharded step on one GPU (compute side)" % W,
        "value": t1 / (W * tmax), "unit": "predicted compute efficiency t1 / (W * max_r t_r)",
        "n_gpus": 1, "rehearsed_world": W, "steps": steps, "warmup": warmup,
        "higher_is_better": True, "dtype": dtype,
        "config": {"workload": "%d ch x 2^%d x %d DM (%g-%g pc/cc), %d time batches, pieces "
                               "layout (P = N / (batches * W) = %d)"
                               % (C, int(np.log2(N)), D, cfg["dm_lo"], cfg["dm_hi"], nb,
                                  N // (nb * W)),
                   "config_name": args.config, "dms_per_trial_block": db},
        "one_gpu": {"step_ms": t1, "sweep_kernel_ms": k1, "launches": l1,
                    "outside_stage2_ms": t1 - k1, "fx": list(fx1)},
        "ranks": ranks,
        "max_rank_step_ms": tmax,
        "mean_rank_step_ms": float(np.mean([x["step_ms"] for x in ranks])),
        "max_over_mean": tmax / float(np.mean([x["step_ms"] for x in ranks])),
        "predicted_step_ms_at_W": tmax,
        "note": "all-gathers replaced by a pre-filled block: exchange time excluded "
                "(DESIGN.md §5 models it: batch k+1's all-gather overlaps batch k's sweep, "
                "only the first batch's is exposed)",
    }
    from pypulsar_amd.delays import sweep_table
    n_out = N - int(sweep_table(dms[-1:], freqs, dt).max())
    line["predicted_value_at_W"] = D * n_out * C / (tmax * 1e-3)
    print(json.dumps(line), flush=True)


def rehearse_timeshard(args, cfg, dev):
    """The W-rank TIME-sharded step rehearsed on ONE GPU: first the whole
    block as one rank (W = 1: the whole plane), then rank r = 0..W-1 exactly
    as it runs in a W-GPU job (TimeShardedSweep(world=W, rank=r): corner turn
    of its own input spectra -- its plane columns plus the max-delay overlap
    -- and the sweep of the whole grid over its columns).  There is no
    exchange to replace: the rank's compute IS its W-GPU step (inputs
    resident).  Reports per-rank step and sweep-kernel times and the
    predicted efficiency t(1 GPU) / (W * max_r t_r)."""
    from pypulsar_amd.sharding import TimeShardedSweep
    W = args.rehearse
    C, N, D = cfg["C"], cfg["N"], cfg["D"]
    dtype = args.dtype or cfg["dtype"]
    tdt = torch.uint8 if dtype == "u8" else torch.float32
    dt = 64e-6
    freqs = band(C)
    dms = np.linspace(cfg["dm_lo"], cfg["dm_hi"], D)
    steps = args.steps if args.steps is not None else 3
    warmup = args.warmup if args.warmup is not None else 1
    block = synth_block(N, C, 1000, dtype, dev)            # time-major [N, C], file order

    def timed(ts, part):
        for _ in range(warmup):
            ts(part)
        torch.cuda.synchronize()
        ts.sw.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            ts(part)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        kms, launches = ts.sw.timing_read()
        ts.sw.set_timing(False)
        return el, kms / steps, launches // steps

    res = []
    # ONE copy stream for every rehearsed rank, as each rank process of a
    # W-GPU job has: a new torch stream per rank eventually shares a hardware
    # queue with the compute stream (4 per process) and its H2D chunks then
    # serialise behind the sweep (the 7th stream of a process: +28 ms)
    cs = torch.cuda.Stream(device=dev)
    for w, r in [(1, 0)] + [(W, r) for r in range(W)]:
        ts = TimeShardedSweep(dms, freqs, dt, N, dtype=tdt, world=w, rank=r, device=dev,
                              factor=_factor_arg(args))
        lo, hi = ts.input_range()
        t, k, l = timed(ts, block[lo:hi])
        g, npat = ts.sw.factor_info(1 if dtype == "u8" else 0)
        rec = {"rank": r, "world": w, "cols": [ts.a, ts.b], "input": [lo, hi],
               "step_ms": t, "sweep_kernel_ms": k, "launches": l, "fx": [g, npat]}
        if not args.no_e2e:
            # the same rank step from its input in pinned host memory
            # (TimeShardedSweep.host_step: chunked H2D under the column ranges)
            hpart = torch.empty((hi - lo, C), dtype=tdt, pin_memory=True)
            hpart.copy_(block[lo:hi])
            e2e = []
            ts.host_step(hpart, n_batches=4, copy_stream=cs)  # (untimed: first-touch of the path)
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ts.host_step(hpart, n_batches=4, copy_stream=cs)
                torch.cuda.synchronize()
                e2e.append((time.perf_counter() - t0) * 1e3)
            h = torch.empty((hi - lo, C), dtype=tdt, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h.copy_(hpart, non_blocking=True)
            torch.cuda.synchronize()
            rec["e2e_step_ms"] = min(e2e)
            rec["h2d_ms"] = (time.perf_counter() - t0) * 1e3
            rec["h2d_bytes"] = hpart.numel() * hpart.element_size()
            del hpart, h
        res.append(rec)
        log("rehearse timeshard: W=%d rank %d columns [%d, %d) step %.1f ms (sweep %.1f ms, "
            "%d launches; PCIe-inclusive %s ms)" % (w, r, ts.a, ts.b, t, k, l,
                                                    rec.get("e2e_step_ms")))
        n_out = ts.n_out
        ts.close()
        del ts
        torch.cuda.empty_cache()
    one, ranks = res[0], res[1:]
    tmax = max(x["step_ms"] for x in ranks)
    line = {
        "metric": "rehearsal of the %d-GPU time-sharded step on one GPU" % W,
        "value": one["step_ms"] / (W * tmax),
        "unit": "predicted efficiency t1 / (W * max_r t_r)",
        "n_gpus": 1, "rehearsed_world": W, "steps": steps, "warmup": warmup,
        "higher_is_better": True, "dtype": dtype,
        "config": {"workload": "%d ch x 2^%d x %d DM (%g-%g pc/cc), time-sharded: rank r sweeps "
                               "plane columns [a_r, b_r) from input spectra [a_r, b_r + max delay)"
                               % (C, int(np.log2(N)), D, cfg["dm_lo"], cfg["dm_hi"]),
                   "config_name": args.config, "mode": "timeshard"},
        "one_gpu": one, "ranks": ranks,
        "max_rank_step_ms": tmax,
        "mean_rank_step_ms": float(np.mean([x["step_ms"] for x in ranks])),
        "predicted_step_ms_at_W": tmax,
        "predicted_value_at_W": D * n_out * C / (tmax * 1e-3),
        "note": "no exchange exists in this partition (each rank's input spectra are its own "
                "H2D); the rank steps are the W-GPU step's per-rank compute exactly",
    }
    if not args.no_e2e:
        emax = max(x["e2e_step_ms"] for x in ranks)
        line["pcie_inclusive"] = {
            "one_gpu_step_ms": one["e2e_step_ms"], "max_rank_step_ms": emax,
            "predicted_efficiency": one["e2e_step_ms"] / (W * emax),
            "median_rank_step_ms": float(np.median([x["e2e_step_ms"] for x in ranks])),
            "predicted_value_at_W": D * n_out * C / (emax * 1e-3),
            "note": "each rank's step from its input spectra in pinned host memory "
                    "(TimeShardedSweep.host_step: 4 H2D chunks on a copy stream under 4 column "
                    "ranges, chunk 0 exposed), rehearsed one rank at a time on one GPU: the "
                    "W ranks' concurrent H2D streams (one PCIe Gen5 x16 link per GPU, a shared "
                    "host memory) are not contended here"}
    print(json.dumps(line), flush=True)


def _finish(args, world, line):
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def ops_bench(args, cfg, rank, world, dev):
    """HBM roofline of the single-DM kernels (read the input
    once + write the output once = the algorithmic bytes) on a C x N block
    resident in HBM, each timed with HIP events on the stream it runs on
    (torch's current stream), mean of --steps launches after --warmup; and
    BASELINE.json configs[0] -- Spectra.dedisperse(100, padval, trim=True) +
    channel sum of a 1024 x 2^16 8-bit filterbank -- through the drop-in
    Spectra API (device-resident data), with the NumPy oracle of the same
    call on one host core beside it.  Rank-local: every rank measures its own
    GPU (no collective in this mode); rank 0 prints."""
    from pypulsar_amd import _lib
    from pypulsar_amd._lib import call, ptr, stream_ptr
    from pypulsar_amd.formats.spectra import Spectra
    C, N = cfg["C"], cfg["N"]
    x8t = synth_block(N, C, 7 + rank, "u8", dev)           # [N, C] filterbank order
    x8 = x8t.t().contiguous()                              # [C, N] raw bytes
    xf = x8.float()                                        # [C, N] float32
    freqs = band(C)
    from pypulsar_amd.delays import dedisperse_bins
    bins = torch.from_numpy(np.asarray(dedisperse_bins(1000.0, freqs, 64e-6), dtype=np.int32)).to(dev)
    zero = torch.zeros(C, dtype=torch.float32, device=dev)
    o_cn = torch.empty((C, N), dtype=torch.float32, device=dev)
    o_ds = torch.empty((C, N // 4), dtype=torch.float32, device=dev)
    o_zt = torch.empty((N, C), dtype=torch.uint8, device=dev)
    o_sub = torch.empty((64, N), dtype=torch.float32, device=dev)
    o_ser = torch.empty((1, N), dtype=torch.float32, device=dev)
    o_c = torch.empty(C, dtype=torch.float32, device=dev)
    o_zd = torch.empty((C, N // 2), dtype=torch.float32, device=dev)
    st = stream_ptr()
    F, U8 = _lib.F32, _lib.U8
    cn4, cn1 = C * N * 4, C * N
    ops = [
        ("shift_pad (dedisperse, pad 0)", "Spectra.shift_channels spectra.py:54-94", cn4 + cn4,
         lambda: call("pdd_shift_pad", ptr(xf), C, N, N, ptr(bins), _lib.PAD_VALUE, ptr(zero),
                      ptr(o_cn), N, N, st)),
        ("shift_group_sum nsub=1 (dedispersed series)", "dedisperse + waterfaller.py:140",
         cn4 + N * 4,
         lambda: call("pdd_shift_group_sum", ptr(xf), C, N, N, ptr(bins), _lib.PAD_VALUE,
                      ptr(zero), 1, ptr(o_ser), N, N, st)),
        ("shift_group_sum nsub=64 (subband)", "Spectra.subband spectra.py:96-138",
         cn4 + 64 * N * 4,
         lambda: call("pdd_shift_group_sum", ptr(xf), C, N, N, ptr(bins), _lib.PAD_VALUE,
                      ptr(zero), 64, ptr(o_sub), N, N, st)),
        ("downsample f32 x4", "Spectra.downsample spectra.py:329-351", cn4 + cn4 // 4,
         lambda: call("pdd_downsample", ptr(xf), C, N, N, 4, ptr(o_ds), N // 4, st)),
        ("downsample u8 x4", "Spectra.downsample (raw 8-bit rows)", cn1 + cn4 // 4,
         lambda: call("pdd_downsample_u8", ptr(x8), C, N, N, 4, ptr(o_ds), N // 4, st)),
        ("zero_dm u8 time-major (wrap)", "zero_dm_filter.py:30-50", cn1 + cn1,
         lambda: call("pdd_zero_dm", ptr(x8t), U8, N, C, C, _lib.LAYOUT_TIME_MAJOR, ptr(o_zt),
                      C, st)),
        ("corner_turn u8 [N,C] -> f32 [C,N]", "filterbank.get_spectra .T + astype",
         cn1 + cn4,
         lambda: call("pdd_corner_turn", ptr(x8t), U8, N, C, C, ptr(o_cn), F, N, st)),
        ("zdm_downsample u8 x2 (stream prologue)", "zero-DM + downsample + corner turn",
         cn1 + cn4 // 2,
         lambda: call("pdd_zdm_downsample", ptr(x8t), U8, N, C, C, 2, 1, ptr(o_zd), N // 2,
                      st)),
        ("channel_stats mean", "shift_channels padval='mean' spectra.py:83-86", cn4 + C * 4,
         lambda: call("pdd_channel_stats", ptr(xf), C, N, N, _lib.STAT_MEAN, ptr(o_c), st)),
        ("smooth width 8", "Spectra.smooth spectra.py:262-303", cn4 + cn4,
         lambda: call("pdd_smooth", ptr(xf), C, N, N, 8, _lib.PAD_VALUE, ptr(zero), ptr(o_cn),
                      N, st)),
    ]
    rows = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, ref, nbytes, fn in ops:
        for _ in range(max(1, args.warmup)):
            fn()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(args.steps):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / args.steps
        gbs = nbytes / (ms * 1e-3) / 1e9
        rows.append({"kernel": name, "reference": ref, "bytes": nbytes, "ms": ms,
                     "achieved_GBs": gbs, "frac_hbm": gbs / PEAK_HBM_GBS})

    # BASELINE.json configs[0] through the drop-in API
    wC, wN, wdm = cfg["wf_C"], cfg["wf_N"], cfg["wf_dm"]
    wfreqs = band(wC)
    w8 = synth_block(wC, wN, 11, "u8", dev)
    wf = {}
    for pad in (0, "mean"):
        def one():
            s = Spectra(wfreqs, 64e-6, w8)  # the reference constructor: u8 -> float copy
            s.dedisperse(wdm, padval=pad, trim=True)
            return s.sum_channels()
        for _ in range(3):
            one()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ser = one()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        wf["padval_%s" % pad] = {"ms": ms, "n_out": int(ser.shape[-1])}
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle import spectra_oracle as orc
        xh = w8.cpu().numpy().astype(np.float64)
        cpu = {}
        for pad in (0, "mean"):
            t0 = time.perf_counter()
            out, _ = orc.dedisperse(xh, wfreqs, 64e-6, wdm, padval=pad, trim=True)
            out.sum(axis=0)
            cpu["padval_%s" % pad] = {"ms": (time.perf_counter() - t0) * 1e3}
        cpu.update({"cores": 1, "kind": "port", "cpu_model": _cpu_model(),
                    "sample": "the same call on the same block (float64 NumPy, C-order, 1 thread)"})
    if rank == 0:
        line = {"metric": "HBM roofline of the single-DM kernels (algorithmic bytes / kernel time)",
                "value": float(np.mean([r["frac_hbm"] for r in rows])),
                "unit": "mean fraction of 8 TB/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "higher_is_better": True, "dtype": "f32/u8",
                "data": "synthetic (uint8 clip(round(N(128,16))), generated on device)",
                "config": {"workload": "single-DM ops on %d ch x 2^%d samples (DM 1000 shifts, "
                                       "1250-1550 MHz, 64 us); configs[0] waterfaller "
                                       "dedisperse %d ch x 2^%d at DM %g"
                                       % (C, int(np.log2(N)), wC, int(np.log2(wN)), wdm),
                           "config_name": "ops"},
                "ops": rows, "waterfaller_config0": {"gpu": wf, "cpu_baseline": cpu}}
        print(json.dumps(line))


def search_bench(args, cfg, rank, world, dev):
    """Single-pulse boxcar search (pypulsar_amd.search) of the config2 DM-time
    plane (1024 DMs x 1,034,083 samples, f32, made once by the sweep, untimed).
    One step = chunk statistics + boxcar search of the whole plane, 13 widths
    1..150.  Both kernels read the plane once: algorithmic bytes per step =
    2 x plane bytes (+ the per-chunk stats, <0.1%)."""
    from pypulsar_amd.search import SinglePulseSearch
    from pypulsar_amd.sweep import DMSweep
    C, N, D = cfg["C"], cfg["N"], cfg["D"]
    dt = 64e-6
    dms = np.linspace(cfg["dm_lo"], cfg["dm_hi"], D)
    sw = DMSweep(dms, band(C), dt, dtype="u8")
    x = synth_block(C, N, 1234 + rank, "u8", dev)
    plane = sw(x, trim=True)
    del x
    sps = SinglePulseSearch(threshold=6.0)
    n = plane.shape[1]
    for _ in range(args.warmup):
        sps.raw(plane)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    for _ in range(args.steps):
        cands, count = sps.raw(plane)
    ev[1].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        el = max_over_ranks(el, dev)
    ms = ev[0].elapsed_time(ev[1]) / args.steps
    byts = 2 * D * n * 4
    achieved = byts / (ms * 1e-3) / 1e9
    line = {
        "metric": "DM-time plane samples searched/sec (single-pulse boxcar search)",
        "value": D * n * world * args.steps / el,
        "unit": "plane samples/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "config2 sweep plane of a synthetic uint8 filterbank (generated on device)",
        "config": {"workload": "boxcar search of a %d DM x %d sample plane, widths 1..150 (13), "
                               "detrend chunks 1000, threshold 6" % (D, n),
                   "candidates_last_step": int(count.item())},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                     "kernel": "pdd::k_sp_stats + pdd::k_sp_search", "kernel_ms": ms,
                     "bytes_per_step": byts},
        "cpu_baseline": None,
    }
    return _finish(args, world, line)


def stream_bench(args, cfg, rank, world, dev):
    """BASELINE configs[4]: continuous 8-bit blocks [block, C] from PINNED host
    memory -> async H2D (copy stream) -> fused zero-DM + downsample 2 ->
    2048-DM sweep (pypulsar_amd.stream; default zero-DM mode 'wrap': the
    reference's uint8 result, (x - round(mean)) mod 256, swept exactly on the
    16-bit path; --zdm float for the float32 path).  One step = one block through the
    whole pipeline, H2D included.  Each rank streams its own data (weak).
    roofline: the block's pinned H2D against this box's pinned H2D rate (the
    binding resource); roofline.sweep_kernel: the sweep kernel's own LDS
    fraction in the adds it performs; cpu_baseline: the oracle's prologue +
    trials on a bounded slice (stream_cpu_baseline)."""
    from pypulsar_amd import _lib
    from pypulsar_amd.stream import StreamingSweep
    C, D, ds = cfg["C"], cfg["D"], cfg["ds"]
    block = args.block or cfg["N"]
    dt = 64e-6
    freqs = band(C)
    dms = np.linspace(cfg["dm_lo"], cfg["dm_hi"], D)
    if args.search:
        from pypulsar_amd.search import StreamingSearch
        ss = StreamingSearch(dms, freqs, dt, block=block, downsamp=ds, threshold=8.0,
                             detrendlen=1024, zero_dm=args.zdm)
        st = ss.sweep
    else:
        st = StreamingSweep(dms, freqs, dt, block=block, downsamp=ds, zero_dm=args.zdm)
    # two distinct pinned chunks, reused cyclically (content is irrelevant to speed)
    chunks = []
    for i in range(2):
        x = synth_block(block, C, 2000 + 10 * rank + i, "u8", dev)
        h = torch.empty((block, C), dtype=torch.uint8, pin_memory=True)
        h.copy_(x)
        chunks.append(h)
    del x
    torch.cuda.synchronize()
    nb = st.n_out_block
    planes = [torch.empty((D, nb), dtype=torch.float32, device=dev) for _ in range(3)]
    total = args.warmup + args.steps + 1  # +1: a block is emitted when the next chunk arrives
    if args.search:  # searched one block behind the sweep
        gen = ss((chunks[i % 2] for i in range(total + 1)), planes=planes)
    else:
        gen = st((chunks[i % 2] for i in range(total)), planes=planes)
    done = 0
    t0 = None
    ncand = 0
    for item in gen:
        if args.search:
            ncand += len(item)
        done += 1
        if done == args.warmup:
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            # the sweep kernel's own launches, timed by the plan's HIP event
            # pairs on the stream it runs on (its LDS fraction below)
            st.sweep.set_timing(True, code=_lib.U16 if st.exact else _lib.F32)
            t0 = time.perf_counter()
        if done == args.warmup + args.steps:
            break
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    k_ms, k_n = st.sweep.timing_read()
    st.sweep.set_timing(False, code=_lib.U16 if st.exact else _lib.F32)
    if world > 1:
        el = max_over_ranks(el, dev)
    units = D * nb * C * args.steps * world
    value = units / el
    lds_roof = N_CU * CLK_GHZ * 1e9 * LDS_B_PER_CLK / 16 * (8 if st.exact else 4) / 1e12
    ms = el / args.steps * 1e3
    in_rate = block * args.steps * world / el  # input spectra per second
    fx_g, fx_pat = st.sweep.factor_info(2 if st.exact else 0) if st.exact else (0, 0)
    h2d_bytes = block * C  # one 8-bit block per step over PCIe (pinned, async)
    # the binding resource: the block's pinned H2D, against this box's own
    # pinned H2D rate (the same bytes copied alone, best of 5)
    h2d_peak = _pinned_h2d_GBs(chunks[0], dev)
    h2d_at = h2d_bytes / (ms * 1e-3) / 1e9
    # the sweep kernel alone: factorised adds per launch over its HIP-event time
    k_adds = D * nb * C / max(1, fx_g)
    k_launch_ms = k_ms / k_n if k_n else None
    k_tadds = k_adds / (k_launch_ms * 1e-3) / 1e12 if k_launch_ms else None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = stream_cpu_baseline(C, ds, dms, dt, nb, D, st.mode)
    line = {
        "metric": "DM-trial samples*channels/sec (node) + % HBM roofline",
        "value": value, "unit": "samples*channels*DM/s (downsampled samples)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic uint8 clip(round(N(128,16))) blocks in pinned host memory",
        "config": {"workload": "streaming: %d-ch u8 blocks of %d spectra (pinned H2D, async) + "
                               "zero-DM (%s) + downsample %d + %d-DM sweep (0-%g pc/cc, %s)%s"
                               % (C, block, st.mode, ds, D, cfg["dm_hi"],
                                  "exact u16" if st.exact else "float32",
                                  " + boxcar search (13 widths, S/N 8)" if args.search else ""),
                   "candidates": ncand if args.search else None,
                   "zero_dm_semantics": {"wrap": "the reference's own: uint8 (x - round(mean)) "
                                                 "mod 256, zero_dm_filter.py:30-39",
                                         "int": "the reference's rounding without the uint8 wrap",
                                         "float": "x - mean in float32 (the reference's float "
                                                  "data semantics)",
                                         "none": "no filter"}[st.mode],
                   "u16_flush_channels": (min(256, 65535 // (st.input_max * max(1, fx_g)))
                                          if st.exact else None),
                   "method": ("exact factorisation over groups of %d channels (%d pattern "
                              "series; plane bit-identical)" % (fx_g, fx_pat) if fx_g
                              else "channel by channel"),
                   "config_name": "stream", "channels": C, "block": block, "overlap": st.ov,
                   "downsamp": ds, "dm_trials": D, "parallelism": "tb%d" % world},
        "realtime_factor": (block * dt) / (ms * 1e-3),
        "input_spectra_per_s": in_rate,
        "roofline": {"bound": "pcie", "achieved": h2d_at, "peak": h2d_peak, "unit": "GB/s",
                     "frac": h2d_at / h2d_peak if h2d_peak else None, "traffic": None,
                     "kernel": "pinned H2D of the 8-bit block (hipMemcpyAsync on the copy "
                               "stream)",
                     "note": "the step's binding resource: one %d-byte block per step over "
                             "PCIe; peak = this box's pinned H2D rate for the same bytes "
                             "copied alone (best of 5); the prologue and the sweep run under "
                             "the copy (sweep_kernel)" % h2d_bytes,
                     "sweep_kernel": {
                         "kernel": "pdd::k_sweep_il (%s)" % ("factorised stage 2, groups of %d"
                                                             % fx_g if fx_g else
                                                             ("u16 eighths" if st.exact else
                                                              "float32 quarters")),
                         "bound": "lds", "unit": "T adds/s", "peak": lds_roof,
                         "ms_per_launch": k_launch_ms, "launches_per_step": k_n / args.steps,
                         "adds_per_launch": k_adds, "achieved": k_tadds,
                         "frac": k_tadds / lds_roof if k_tadds else None,
                         "note": "adds the kernel performs (D x columns x C / g) over its own "
                                 "HIP-event time; 8-bit factorised adds read 2 B of LDS each"}},
        "h2d_bytes_per_step": h2d_bytes,
        "h2d_GBs_at_step": h2d_at,
        "cpu_baseline": cpu,
    }
    st.close()
    _finish(args, world, line)


def subband_bench(args, cfg, rank, world, dev):
    """BASELINE configs[2]: two-stage subband dedispersion over the DDplan2b
    grid (Observation(64us, 1400, 300, 4096).gen_ddplan(0, 1000, 64, 0.5)):
    per DDstep downsample, then all 40 subband passes as ONE grouped sweep
    (stage 1) and all passes' DM sweeps as ONE grouped sweep (stage 2)
    (pypulsar_amd.sweep.DDplanExecutor, plans built once; equal to the per-pass
    subband(64, subDM) + sweep executor, tests/test_gpu_grouped.py).  Work
    units are the equivalent brute-force samples*channels*DM of the plan's
    trials (the quantity the two-stage method replaces)."""
    from pypulsar_amd.formats.spectra import Spectra
    from pypulsar_amd.sweep import DDplanExecutor
    from pypulsar_amd.utils.ddplan import Observation
    C, N = cfg["C"], cfg["N"]
    dt = 64e-6
    freqs = band(C)
    plan = Observation(dt, 1400.0, 300.0, C).gen_ddplan(cfg["dm_lo"], cfg["dm_hi"], cfg["nsub"],
                                                       cfg["res"])
    x = synth_block(C, N, 3000 + rank, "u8", dev)
    s = Spectra(freqs, dt, x)
    units = 0
    for step in plan.DDsteps:
        n_ds = N // step.downsamp
        from pypulsar_amd.delays import sweep_table
        mb = int(max(0, sweep_table(step.DMs[-1:], freqs, dt * step.downsamp).max()))
        units += len(step.DMs) * (n_ds - mb) * C

    # delay tables, grouped plans and buffers built once per grid
    ex = DDplanExecutor(plan, freqs, dt, N, raw8=True)

    def one():
        return ex(s, padval=0)

    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        el = max_over_ranks(el, dev)
    ms = el / args.steps * 1e3
    roof = subband_roofline(ex, s, one, args.steps, C, N) if world == 1 else None
    line = {
        "metric": "DM-trial samples*channels/sec (node) + % HBM roofline",
        "value": units * args.steps * world / el,
        "unit": "samples*channels*DM/s (brute-force-equivalent)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic uint8 clip(round(N(128,16))) filterbank, generated on device",
        "config": {"workload": "two-stage subband sweep %d ch -> %d subbands, DDplan2b "
                               "(0-%g pc/cc, res %g ms): %s" % (C, cfg["nsub"], cfg["dm_hi"],
                                                               cfg["res"],
                                                               [(len(st.DMs), st.downsamp,
                                                                 st.numprepsub)
                                                                for st in plan.DDsteps]),
                   "config_name": "subband", "channels": C, "samples": N,
                   "dm_trials": int(sum(len(st.DMs) for st in plan.DDsteps)),
                   "parallelism": "tb%d" % world},
        "roofline": roof,
        "cpu_baseline": None,
    }
    _finish(args, world, line)


def subband_roofline(ex, spectra, one, steps, C, N):
    """Per-stage roofline of a chained two-stage DDplan step (configs[2]:
    pdd_subband_chain = the stage-1 interleave pre-pass (8-bit rows co-added
    by ds into u16 eighths), the stage-1 grouped sweep writing stage 2's
    float32 quarters image, the stage-2 grouped sweep writing the plane).
    The two sweep kernels are timed by their plans' HIP event pairs, the
    whole chain by events around it on the same stream; the pre-pass is the
    remainder.  Each stage is priced against its own bound: the pre-pass
    against HBM (its input once + its output once), the sweeps against the
    LDS read roof of their image (u16 eighths: 2 B per add; float32
    quarters: 4 B per add) in the adds of the plan's REAL trials (the tile's
    padded trial slots are not counted), with their HBM fractions beside.
    None unless the chained u16 stage 1 ran (8-bit rows, integer pads:
    otherwise stage 1 is a float32 sweep and its timers read 0)."""
    st = [s for s in ex.steps if s.two_stage and s.chain]
    if len(ex.steps) != 1 or not st:
        return None
    s = st[0]
    if s.int1 != "u16":
        return None
    i1, i2 = s.g1.info(), s.g2.info()
    n1 = N // s.ds
    tq = i1["samples_per_block"] // 8                   # u16 eighths: Tq elements
    qs1 = -(-(-(-n1 // 8)) // tq) * tq
    nr1 = qs1 + max(0, i1["max_bin"]) - min(0, i1["min_bin"]) + 64
    rows2 = s.ncall * s.nsub
    nr2 = 2 * qs1 + max(0, i2["max_bin"]) + 64
    b_pre = C * N + C * nr1 * 16                         # raw 8-bit rows in, u16 eighths out
    b_s1 = C * nr1 * 16 + rows2 * nr2 * 16               # eighths in, quarters image out
    b_s2 = rows2 * nr2 * 16 + s.ncall * s.per * s.n_out * 4   # quarters in, plane out
    cps = C // s.nsub
    adds1 = s.nsub * s.ncall * cps * n1                  # every subband sample of every pass
    adds2 = s.ncall * s.per * s.nsub * s.n_out           # every plane sample of every DM
    s.g1.set_timing(True)
    s.g2.set_timing(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        one()
    e1.record()
    torch.cuda.synchronize()
    t_all = e0.elapsed_time(e1) / steps
    k1, l1 = s.g1.timing_read()
    k2, l2 = s.g2.timing_read()
    s.g1.set_timing(False)
    s.g2.set_timing(False)
    if not (l1 and l2 and k1 > 0 and k2 > 0):
        return None
    k1, k2 = k1 / steps, k2 / steps
    pre = max(t_all - k1 - k2, 1e-6)
    lds_u16 = N_CU * CLK_GHZ * 1e9 * LDS_B_PER_CLK / 2 / 1e12    # T adds/s, 2 B per add
    lds_f32 = lds_u16 / 2
    stages = []
    for name, b, t, adds, roof, db in (
            ("k_interleave_u16_ds_v (stage-1 pre-pass: co-add + eighths)", b_pre, pre, None,
             None, None),
            ("k_sweep_il u16 grouped, stage 1 -> stage-2 quarters image", b_s1, k1, adds1,
             lds_u16, i1["dms_per_block"]),
            ("k_sweep_il f32 grouped, stage 2 -> plane", b_s2, k2, adds2, lds_f32,
             i2["dms_per_block"])):
        gbs = b / (t * 1e-3) / 1e9
        e = {"kernel": name, "ms": t, "bytes": b, "achieved_GBs": gbs,
             "hbm_frac": gbs / PEAK_HBM_GBS}
        if adds is None:
            e.update(bound="hbm", frac=gbs / PEAK_HBM_GBS)
        else:
            ta = adds / (t * 1e-3) / 1e12
            trials = s.ncall if "stage 1" in name else s.per
            e.update(bound="lds", adds=adds, achieved_Tadds=ta, lds_peak_Tadds=roof,
                     frac=ta / roof, trials_per_group=trials, tile_trials=db,
                     tile_fill=trials / (-(-trials // db) * db))
        stages.append(e)
    dom = max(stages, key=lambda e: e["ms"])
    return {"bound": dom["bound"], "achieved": dom.get("achieved_Tadds", dom["achieved_GBs"]),
            "peak": dom.get("lds_peak_Tadds", PEAK_HBM_GBS),
            "unit": "T adds/s" if dom["bound"] == "lds" else "GB/s",
            "frac": dom["frac"], "kernel": dom["kernel"], "traffic": None,
            "stages": stages, "launches": [l1 // steps, l2 // steps],
            "chain_ms": t_all,
            "note": "top level = the longest stage against its own bound; each stage: the "
                    "pre-pass against HBM (input once + output once), the sweeps against the "
                    "LDS read roof of their image in the adds of the real trials (padded tile "
                    "slots excluded, tile_fill), with their HBM fractions (hbm_frac)"}

if __name__ == "__main__":
    main()
