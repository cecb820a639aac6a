"""Multi-core CPU baseline runner for the NumPy / literal-loop restatements (ofdm_oracle).

TEST / BASELINE INFRASTRUCTURE ONLY: started by bench.py's cpu_baseline leg as a CHILD
process (so the worker pool forks from a process that never touched the GPU), never part of
the product.

    python oracle/cpu_pool.py <input.npy> <L> <form: numpy|loop> <workers> <budget_s>

Runs ``ofdm_oracle.aa_detect`` (vectorised prefix sums + the reference's gate loop) or
``ofdm_oracle.aa_detect_loop`` (the reference's per-sample streaming loop, sync_aa.py:458-568)
over the streams of x[B, n_ant, T], one stream per task, on a pool of `workers` processes,
until ~budget_s of wall time (cycling over the streams); prints one JSON line with the rate.
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ofdm_oracle as O  # noqa: E402

_X = None


def _init(path):
    global _X
    _X = np.load(path, mmap_mode="r")


def _one(args):
    b, L, form = args
    x = np.asarray(_X[b], dtype=np.complex128)
    (O.aa_detect_loop if form == "loop" else O.aa_detect)(x, L)
    return x.shape[-1]


def main():
    path, L, form, workers, budget = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), float(sys.argv[5])
    X = np.load(path, mmap_mode="r")
    B, T = X.shape[0], X.shape[-1]
    ctx = mp.get_context("fork")
    with ctx.Pool(workers, initializer=_init, initargs=(path,)) as pool:
        pool.map(_one, [(b % B, L, form) for b in range(workers)])          # warm every worker
        done, t0, b = 0, time.perf_counter(), 0
        chunk = workers * (1 if form == "loop" else 8)
        while time.perf_counter() - t0 < budget and b < 64 * B:   # the sample cycles over the streams
            done += sum(pool.map(_one, [(i % B, L, form) for i in range(b, b + chunk)]))
            b += chunk
        dt = time.perf_counter() - t0
    print(json.dumps(dict(value=done / dt / 1e6, streams=b, samples=done, seconds=dt, workers=workers,
                          form=form, T=T)))


if __name__ == "__main__":
    main()
