"""CPU baseline worker (TEST / MEASUREMENT INFRASTRUCTURE, not product code).

``bench.py``'s ``cpu_baseline.all_cores`` leg starts one of these per host
core of the lease as a fresh interpreter (``python -m oracle.cpu_pool``): it
imports only NumPy and the oracle (no torch, so no GPU file descriptors are
inherited and every core of the lease can run one).  Protocol on stdin /
stdout, one JSON line each way:

  parent -> worker  {"x": path of a [C, n] float64 .npy, "freqs": [...],
                     "dt": s, "tasks": [[c0, c1, dm, n_keep], ...]}
  worker -> parent  "ready"            (block mapped, first task done untimed)
  parent -> worker  "go"
  worker -> parent  {"work": units, "elapsed": s}

Each task is the reference algorithm on one channel block of one DM trial
(oracle.spectra_oracle.shift_channels on rows c0..c1 -- formats/spectra.py:54-94
-- then the channel sum of the first n_keep samples, bin/waterfaller.py:140):
the channel sum of a trial is the sum of its channel-block partial sums.
"""
import json
import sys
import time

import numpy as np


def _run(x, freqs, dt, task, orc):
    c0, c1, dm, n_keep = task
    bins = orc.dedisperse_bins(dm, 0.0, freqs, dt)
    sub = orc.shift_channels(np.array(x[c0:c1]), bins[c0:c1], padval=0)
    sub[:, :n_keep].sum(axis=0)
    return (c1 - c0) * n_keep


def main():
    from oracle import spectra_oracle as orc
    spec = json.loads(sys.stdin.readline())
    x = np.load(spec["x"], mmap_mode="r")
    freqs = np.asarray(spec["freqs"], dtype=np.float64)
    tasks = spec["tasks"]
    if tasks:
        _run(x, freqs, spec["dt"], tasks[0], orc)  # page in + warm up, untimed
    print("ready", flush=True)
    if sys.stdin.readline().strip() != "go":
        return
    t0 = time.perf_counter()
    work = sum(_run(x, freqs, spec["dt"], t, orc) for t in tasks)
    print(json.dumps({"work": work, "elapsed": time.perf_counter() - t0}), flush=True)


if __name__ == "__main__":
    main()
