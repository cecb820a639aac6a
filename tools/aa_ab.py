"""A/B timing of the headline kernel (ofs_aa_detect, cfg3 shape) with parts switched off, to
see where the time goes: events on/off, outputs stored or not.  Diagnostic only.

    OFS_LIB=build/libofdmsync_x.so python tools/aa_ab.py [--steps K]
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
if os.environ.get("OFS_LIB"):   # a tools/variants.py tuning build, named explicitly (not a product switch)
    _lib.use_tuning_library(os.environ["OFS_LIB"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--realloc", type=int, default=0, help="only the full case, re-allocating all buffers N times")
    ap.add_argument("--same", action="store_true", help="realloc sweep without re-allocating (time variation)")
    ap.add_argument("--contig", action="store_true", help="arena rounds use a physically contiguous arena (bench.py)")
    ap.add_argument("--pre", type=float, default=0.0, help="GiB allocated (and held) before the first round")
    ap.add_argument("--check", action="store_true", help="realloc: compare every library's events")
    ap.add_argument("--libs", default="", help="comma list of library paths timed on the same buffers (realloc)")
    a = ap.parse_args()
    if a.realloc:
        return realloc_sweep(a)
    dev = torch.device("cuda", 0)
    B, T, L, E = a.B, a.T, a.L, 4
    x = synth.make_aa_batch(B, T, L, seed=2026, device=dev)
    P = torch.empty((B, T), dtype=torch.complex64, device=dev)
    R = torch.empty((B, T), dtype=torch.float32, device=dev)
    M = torch.empty((B, T), dtype=torch.float32, device=dev)
    n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    lib = _lib.lib()
    st = torch.cuda.current_stream(dev)
    lib_name = os.path.basename(os.environ.get("OFS_LIB", "default"))
    for name, det, outs in (("full", 1, True), ("no_events", 0, True), ("no_outputs", 1, False),
                            ("read_only", 0, False), ("full_again", 1, True)):
        p = (P.data_ptr(), R.data_ptr(), M.data_ptr()) if outs else (None, None, None)
        args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, *p, None, det, 0.15, 128, 15.36e6, E,
                n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
        fn = lib.ofs_aa_detect
        for _ in range(a.warmup):
            fn(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            rc = fn(*args)
        e1.record(st)
        torch.cuda.synchronize()
        if rc:
            raise RuntimeError(rc)
        ms = e0.elapsed_time(e1) / a.steps
        nbytes = B * T * (24 if outs else 8)
        print(json.dumps({"lib": lib_name, "case": name, "ms": round(ms, 5),
                          "GBs": round(nbytes / ms / 1e6, 1)}), flush=True)


def realloc_sweep(a):
    """Same launch, fresh buffers each round: separates allocation (physical placement) effects
    from code effects."""
    dev = torch.device("cuda", 0)
    B, T, L, E = a.B, a.T, a.L, 4
    import ctypes
    libs = []
    for path in (a.libs.split(",") if a.libs else [_lib.LIB_PATH]):
        l = ctypes.CDLL(os.path.abspath(path))
        _lib._declare(l)
        libs.append((os.path.basename(path), l))
    st = torch.cuda.current_stream(dev)
    keep = []
    pre = torch.empty(int(a.pre * (1 << 30)), dtype=torch.uint8, device=dev) if a.pre > 0 else None
    for r in range(a.realloc):
        if a.same and keep:
            x, P, R, M = keep[0]
            keep.append(keep[0])
            n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
        else:
            if r % 2 == 1:                       # odd rounds: one arena (bench.py layout)
                x, P, R, M = _lib.arena(dev, [((B, 1, T), torch.complex64), ((B, T), torch.complex64),
                                              ((B, T), torch.float32), ((B, T), torch.float32)],
                                             contiguous=a.contig)
                x.copy_(synth.make_aa_batch(B, T, L, seed=2026, device=dev))
            else:
                x = synth.make_aa_batch(B, T, L, seed=2026, device=dev)
                P = torch.empty((B, T), dtype=torch.complex64, device=dev)
                R = torch.empty((B, T), dtype=torch.float32, device=dev)
                M = torch.empty((B, T), dtype=torch.float32, device=dev)
            n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
            ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
            ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
        args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(), None, 1,
                0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
        res = {}
        for name, lib in libs[r % len(libs):] + libs[:r % len(libs)]:     # rotate the order per round
            for _ in range(a.warmup):
                lib.ofs_aa_detect(*args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                lib.ofs_aa_detect(*args)
            e1.record(st)
            torch.cuda.synchronize()
            res[name] = round(e0.elapsed_time(e1) / a.steps, 5)
        res = {n: res[n] for n, _ in libs}
        if a.check:                              # same events from every library (bit-identical)
            outs = []
            for name, lib in libs:
                n_ev.zero_(); ev_i.fill_(-7); ev_r.fill_(-7.0)
                lib.ofs_aa_detect(*args)
                torch.cuda.synchronize()
                outs.append((n_ev.clone(), ev_i.clone(), ev_r.clone()))
            res["events"] = int(outs[0][0].sum())
            res["same"] = all(torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
                              and torch.equal(o[2].view(torch.int64), outs[0][2].view(torch.int64))
                              for o in outs[1:])
        print(json.dumps({"round": r, "ms": res, "x": hex(x.data_ptr()), "P": hex(P.data_ptr())}), flush=True)
        if not a.same or len(keep) == 0:
            keep.append((x, P, R, M))             # hold: the next round gets new physical pages


if __name__ == "__main__":
    main()
