"""Multi-core CPU baseline runner for the NumPy / literal-loop restatements (ofdm_oracle).

TEST / BASELINE INFRASTRUCTURE ONLY: started by bench.py's cpu_baseline leg as a CHILD
process (so the worker pool forks from a process that never touched the GPU), never part of
the product.

    python oracle/cpu_pool.py <input.npy> <L> <form: numpy|loop> <workers> <budget_s>
    python oracle/cpu_pool.py --config <cfg2a|cfg2b|cfg4|cfg5> <workers> <budget_s>

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


# ---- the other BASELINE.json configs: seeded synthetic streams of the config's shape, one
#      stream (or sequence) per task, the NumPy restatement as the CPU path ----------------
CFG = {
    # name: (samples per task, description)
    "cfg2a": (1024, "sync_aa L=128 on int12 I/Q (as complex128), T=1024: ofdm_oracle.aa_detect"),
    "cfg2b": (1024, "minn_rtl Q=64 on int12 I/Q, T=1024, float IIR + threshold + gate: "
                    "ofdm_oracle.minn_rtl_metric + detect_minn_rtl"),
    "cfg4": (4096, "combined_sc_min S&C + Minn, N=2048, T=4096: ofdm_oracle.comb_sc_metric + minn_metric"),
    "cfg5": (4096, "zc_freq 62-bin metric, N=4096, one window per sequence: np.fft per window + 62-bin gather + "
                   "vdot, the reference's loop body (zc_freq.py:85-97)"),
}


def _cfg_task(args):
    name, seed = args
    rng = np.random.default_rng(seed)
    n = CFG[name][0]
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    if name == "cfg2a":
        O.aa_detect(np.round(x * 600.0), 128)
    elif name == "cfg2b":
        st = O.minn_rtl_metric(np.round(x * 600.0), 64, 3, 3276, 15)
        O.detect_minn_rtl(st["corr_positive"], st["above_threshold"], st["metric_valid"], 2, 0)
    elif name == "cfg4":
        O.comb_sc_metric(x, 2048)
        O.minn_metric(x, 2048)
    else:                                   # zc_freq.py:85-97 for the one offset of the sequence
        idx, t, e = O.zc_template()
        N = 4096
        X = np.fft.fftshift(np.fft.fft(x[:N]))
        b = X[(N // 2 + idx) % N]
        _ = np.abs(np.vdot(t, b)) ** 2 / max(e * float(np.sum(np.abs(b) ** 2)), 1e-12)
    return n


def run_config(name, workers, budget):
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        pool.map(_cfg_task, [(name, i) for i in range(workers)])                  # warm
        done, t0, i = 0, time.perf_counter(), 0
        while time.perf_counter() - t0 < budget:
            done += sum(pool.map(_cfg_task, [(name, j) for j in range(i, i + 4 * workers)]))
            i += 4 * workers
        dt = time.perf_counter() - t0
    print(json.dumps(dict(value=done / dt / 1e6, streams=i, samples=done, seconds=dt, workers=workers, config=name,
                          form=CFG[name][1])))


def main():
    if sys.argv[1] == "--config":
        return run_config(sys.argv[2], int(sys.argv[3]), float(sys.argv[4]))
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
