"""Headline batch on physically contiguous backing, three layouts timed in one process and
interleaved: one arena for x|P|R|M (bench.py), x and P|R|M in two contiguous blocks, four
separate contiguous blocks.  Diagnostic only.

    python tools/split_probe.py [--reps R] [--steps K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))

import torch  # noqa: E402

from ofdm_sync_amd import _lib, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    B, T, L, E = 65536, 1024, 512, 4
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    lib = _lib.lib()
    x0 = synth.make_aa_batch(B, T, L, seed=2026, device=dev)
    n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    sx = ((B, 1, T), torch.complex64)
    so = [((B, T), torch.complex64), ((B, T), torch.float32), ((B, T), torch.float32)]

    def layout(name):
        if name == "one":
            return _lib.arena(dev, [sx] + so, contiguous=True)
        if name == "two":
            return _lib.arena(dev, [sx], contiguous=True) + _lib.arena(dev, so, contiguous=True)
        return [_lib.arena(dev, [s], contiguous=True)[0] for s in [sx] + so]

    for rep in range(a.reps):
        for name in ("one", "two", "four"):
            x, P, R, M = layout(name)
            x.copy_(x0)
            args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(), None,
                    1, 0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
            for _ in range(10):
                lib.ofs_aa_detect(*args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                lib.ofs_aa_detect(*args)
            e1.record(st)
            torch.cuda.synchronize()
            print(json.dumps({"rep": rep, "layout": name, "ms": round(e0.elapsed_time(e1) / a.steps, 5)}), flush=True)
            del x, P, R, M
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
