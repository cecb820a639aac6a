"""Paired A/B of libofdmsync.so variants (tools/variants.py) on the same device buffers: the
sync_aa detector (ofs_aa_detect) on one shape, lib order rotated every round.  Diagnostic only.

    python tools/lib_ab.py --libs build/libofdmsync_a.so,build/libofdmsync_b.so --B 65536 --T 4096 --L 512 --na 1
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ofdm_sync_amd import _lib, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--T", type=int, default=4096)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--na", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--detect-only", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="variants may differ in rounding (no bit-equality check)")
    ap.add_argument("--op", choices=("aa", "scminn", "sc", "comb", "minn", "zcfreq"), default="aa",
                    help="aa: ofs_aa_detect; scminn: ofs_sc_minn_metric (cfg4 fused S&C + Minn, N = 2 L); zcfreq: "
                         "ofs_zc_freq_metric on c64 -> f32 (--na branches, N = 4 L, cp = L, the ZC template)")
    a = ap.parse_args()
    if a.op == "zcfreq":
        return zcfreq(a)
    if a.op != "aa":
        return scminn(a)
    dev = torch.device("cuda", 0)
    B, T, L, na, E = a.B, a.T, a.L, a.na, 4
    base = synth.faded_base(L, "cir1", tuple(range(na)) if na > 1 else (1,))
    x = synth.synth_batch(base, B, T, seed=5, device=dev)
    P = None if a.detect_only else torch.empty((B, T), dtype=torch.complex64, device=dev)
    R = None if a.detect_only else torch.empty((B, T), dtype=torch.float32, device=dev)
    M = None if a.detect_only else torch.empty((B, T), dtype=torch.float32, device=dev)
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    libs = []
    for p in a.libs.split(","):
        l = ctypes.CDLL(os.path.abspath(p))
        _lib._declare(l)
        libs.append((os.path.basename(p), l))
    args = (_lib.C64, x.data_ptr(), B, na, T, L, _lib.FP32, _lib.ptr(P), _lib.ptr(R), _lib.ptr(M), None, 1,
            0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
    times = {n: [] for n, _ in libs}
    ref = None
    for r in range(a.rounds):
        order = libs[r % len(libs):] + libs[:r % len(libs)]
        for name, l in order:
            for _ in range(3):
                assert l.ofs_aa_detect(*args) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                l.ofs_aa_detect(*args)
            e1.record(st)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.steps)
            if ref is None:
                ref = (n_ev.clone(), None if M is None else M.clone())
            elif not a.no_check:
                assert torch.equal(ref[0], n_ev), f"{name}: events differ"
                if M is not None:
                    assert torch.equal(ref[1], M), f"{name}: M differs"
    alg = B * T * (na * 8 + (0 if a.detect_only else 16))
    for name, _ in libs:
        ms = statistics.median(times[name])
        print(json.dumps(dict(lib=name, shape=[B, na, T, L], plan=libs[0][1].ofs_aa_plan(_lib.C64, _lib.FP32, na, T, L),
                              ms_median=round(ms, 4), ms_all=[round(t, 4) for t in times[name]],
                              frac=round(alg / (ms / 1e3) / 8e12, 4))), flush=True)


def scminn(a):
    dev = torch.device("cuda", 0)
    B, T, N, nb = a.B, a.T, 2 * a.L, a.na
    x = synth.synth_batch(synth.faded_base(a.L, "cir1", tuple(range(nb)) if nb > 1 else (1,)), B, T, seed=4, device=dev)
    nout = T - N + 1
    n_sets = 2 if a.op == "scminn" else 1
    outs = [torch.empty((B, nout), dtype=dt, device=dev) for dt in (torch.float32, torch.complex64, torch.float32) * n_sets]
    st = torch.cuda.current_stream(dev)
    libs = []
    for p in a.libs.split(","):
        l = ctypes.CDLL(os.path.abspath(p))
        _lib._declare(l)
        libs.append((os.path.basename(p), l))
    optr = [o.data_ptr() for o in outs]
    if a.op == "scminn":
        call = lambda l: l.ofs_sc_minn_metric(_lib.C64, x.data_ptr(), B, nb, T, N, _lib.FP32, *optr, st.cuda_stream)
    elif a.op == "minn":
        call = lambda l: l.ofs_minn_metric(_lib.C64, x.data_ptr(), B, nb, T, N, _lib.FP32, *optr, st.cuda_stream)
    else:
        rm = 0 if a.op == "sc" else 1
        call = lambda l: l.ofs_sc_metric(_lib.C64, x.data_ptr(), B, nb, T, N, rm, _lib.FP32, *optr, st.cuda_stream)
    times = {n: [] for n, _ in libs}
    ref = None
    for r in range(a.rounds):
        for name, l in libs[r % len(libs):] + libs[:r % len(libs)]:
            if not a.no_check:                     # every output element must be rewritten
                for o in outs:
                    o.fill_(float("nan"))
            for _ in range(3):
                assert call(l) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                call(l)
            e1.record(st)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.steps)
            if ref is None:
                ref = [o.clone() for o in outs]
            elif not a.no_check:
                for o, q in zip(outs, ref):
                    assert torch.equal(o, q), f"{name}: outputs differ"
    alg = B * T * 8 * nb + n_sets * B * nout * 16
    for name, _ in libs:
        ms = statistics.median(times[name])
        print(json.dumps(dict(lib=name, op=a.op, shape=[B, nb, T, N], ms_median=round(ms, 4),
                              ms_all=[round(t, 4) for t in times[name]], frac=round(alg / (ms / 1e3) / 8e12, 4))),
              flush=True)


def zcfreq(a):
    """zc_freq on the reference's stream shape by default (--B 4096 --na 2 --T 4242 --L 512: N 2048,
    cp 512); outputs compared within 1e-12 relative (libraries may order the row sums differently)."""
    from ofdm_sync_amd import zc_freq
    dev = torch.device("cuda", 0)
    B, nb, T, N, cp = a.B, a.na, a.T, 4 * a.L, a.L
    g = torch.Generator(device=dev).manual_seed(8)
    x = torch.randn((B, nb, T), dtype=torch.complex64, device=dev, generator=g)
    idx, tb, e = zc_freq.make_pss_frequency_template()
    idx = np.ascontiguousarray(np.asarray(idx, np.int32))
    tb = np.ascontiguousarray(np.asarray(tb, np.complex128))
    noff = T - (N + cp) + 1
    out = torch.empty((B, noff), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev)
    libs = []
    for p in a.libs.split(","):
        l = ctypes.CDLL(os.path.abspath(p))
        _lib._declare(l)
        libs.append((os.path.basename(p), l))
    call = lambda l: l.ofs_zc_freq_metric(_lib.C64, x.data_ptr(), B, nb, T, N, cp, _lib.FP32, int(idx.size),
                                          idx.ctypes.data, tb.ctypes.data, float(e), out.data_ptr(), st.cuda_stream)
    times = {n: [] for n, _ in libs}
    ref = None
    for r in range(a.rounds):
        for name, l in libs[r % len(libs):] + libs[:r % len(libs)]:
            out.fill_(float("nan"))
            for _ in range(3):
                assert call(l) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                call(l)
            e1.record(st)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.steps)
            if ref is None:
                ref = out.double().clone()
            elif not a.no_check:
                d = ((out.double() - ref).abs() / ref.abs().clamp_min(1e-30)).max().item()
                assert d <= 1e-6, f"{name}: metric differs by {d:.3g} relative"
    for name, _ in libs:
        ms = statistics.median(times[name])
        print(json.dumps(dict(lib=name, op=a.op, shape=[B, nb, T, N, cp], ms_median=round(ms, 4),
                              ms_all=[round(t, 4) for t in times[name]])), flush=True)


if __name__ == "__main__":
    main()
