"""ctypes wrapper of oracle/liboracle.so (the C restatement in oracle/csrc/ofs_oracle.c).

TEST / BASELINE INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import c_double, c_int, c_int64, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "csrc", "ofs_oracle.c")
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
            subprocess.run(["gcc", "-O2", "-fopenmp", "-fPIC", "-shared", "-std=c11", "-o", LIB, src, "-lm"],
                           check=True)
        l = ctypes.CDLL(LIB)
        l.oracle_aa_detect.restype = c_int
        l.oracle_aa_detect.argtypes = [c_void_p, c_int, c_int64, c_int64, c_int64, c_int64, c_double,
                                       c_int, c_double, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                       c_void_p, c_void_p, c_int]
        l.oracle_max_threads.restype = c_int
        l.oracle_sc_minn_check.restype = c_int
        l.oracle_sc_minn_check.argtypes = [c_void_p, c_int, c_int64, c_int64, c_int64, c_int64] + [c_void_p] * 6 + \
            [c_int, c_double, c_double, c_double, c_void_p, c_int]
        l.oracle_zc_freq_check.restype = c_int
        l.oracle_zc_freq_check.argtypes = [c_void_p, c_int, c_int64, c_int64, c_int64, c_int64, c_int64, c_int,
                                           c_void_p, c_void_p, c_double, c_void_p, c_int, c_double, c_double,
                                           c_void_p, c_int]
        l.oracle_minn_rtl.restype = c_int
        l.oracle_minn_rtl.argtypes = [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int, c_int64, c_int, c_int,
                                      c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int]
        _lib = l
    return _lib


def aa_detect(x, L, threshold=0.15, hysteresis=128, sample_rate=15.36e6, max_events=16,
              nthreads=0, want_arrays=True):
    """x: [B, n_ant, T] complex64/complex128 (host).  Returns dict of arrays."""
    x = np.ascontiguousarray(x)
    if x.ndim == 2:
        x = x[:, None, :]
    if x.dtype not in (np.complex64, np.complex128):
        x = x.astype(np.complex128)
    B, na, T = x.shape
    P = np.empty((B, T), np.complex128) if want_arrays else None
    R = np.empty((B, T)) if want_arrays else None
    M = np.empty((B, T)) if want_arrays else None
    n_ev = np.zeros(B, np.int32)
    ev_i = np.zeros((B, max_events, 4), np.int64)
    ev_r = np.zeros((B, max_events, 4))
    p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    rc = lib().oracle_aa_detect(x.ctypes.data, int(x.dtype == np.complex128), B, na, T, int(L),
                                float(threshold), int(hysteresis), float(sample_rate), p(P), p(R),
                                p(M), int(max_events), n_ev.ctypes.data, ev_i.ctypes.data,
                                ev_r.ctypes.data, int(nthreads))
    if rc:
        raise RuntimeError(f"oracle_aa_detect failed ({rc})")
    return dict(P=P, R=R, M=M, n_events=n_ev, ev_int=ev_i, ev_real=ev_r)


def minn_rtl(x, Q, smooth_shift=3, threshold_value=3276, threshold_frac_bits=15, hysteresis=2,
             timing_offset=0, max_events=16, nthreads=0):
    """x: [B, nb, T] complex (host) -> dict of the minn_rtl state arrays + detect_minn_rtl events
    (C restatement, float smoothing)."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.complex128))
    if x.ndim == 2:
        x = x[:, None, :]
    B, nb, T = x.shape
    f = lambda: np.empty((B, T))                  # noqa: E731
    u = lambda: np.empty((B, T), np.uint8)        # noqa: E731
    out = dict(corr_total=f(), corr_positive=f(), smooth_metric=f(), energy_total=f(), corr_scaled=f(),
               energy_scaled=f(), metric_valid=u(), above_threshold=u())
    ev = np.zeros((B, max(max_events, 1), 4), np.int64)
    n_ev = np.zeros(B, np.int32)
    og = np.zeros(B, np.int64)
    o = out
    rc = lib().oracle_minn_rtl(x.ctypes.data, B, nb, T, int(Q), int(smooth_shift), int(threshold_value),
                               int(threshold_frac_bits), int(hysteresis), int(timing_offset), int(max_events),
                               o["corr_total"].ctypes.data, o["corr_positive"].ctypes.data,
                               o["smooth_metric"].ctypes.data, o["energy_total"].ctypes.data,
                               o["corr_scaled"].ctypes.data, o["energy_scaled"].ctypes.data,
                               o["metric_valid"].ctypes.data, o["above_threshold"].ctypes.data, ev.ctypes.data,
                               n_ev.ctypes.data, og.ctypes.data, int(nthreads))
    if rc:
        raise RuntimeError(f"oracle_minn_rtl failed ({rc})")
    out.update(events=ev, n_events=n_ev, open_gate_start=og)
    return out


def _host(a, dtype):
    a = np.ascontiguousarray(a)
    if a.dtype != dtype:
        raise TypeError(f"expected {dtype}, got {a.dtype}")
    return a


SC_MINN_STATS = ("comb_max_dM", "comb_dM_over_bound", "comb_dP_over_bound", "comb_dR_over_bound",
                 "minn_max_dM_rel1", "minn_dM_over_bound", "minn_dP_over_bound", "minn_dR_over_bound")


def sc_minn_check(x, N, Mc, Pc, Rc, Mm, Pm, Rm, kP, kR, kM, nthreads=0):
    """Engine combined S&C + Minn outputs ([B, T-N+1]; fp32 / complex64, or fp64 / complex128 for
    all six) against the fp64 reference values of x [B, nb, T] (oracle_sc_minn_check).  Returns the
    per-stream statistics [B, 8] (SC_MINN_STATS)."""
    x = np.ascontiguousarray(x)
    if x.ndim == 2:
        x = x[:, None, :]
    if x.dtype not in (np.complex64, np.complex128):
        raise TypeError("x must be complex64 / complex128")
    B, nb, T = x.shape
    f64 = np.asarray(Mc).dtype == np.float64
    rt, ct = (np.float64, np.complex128) if f64 else (np.float32, np.complex64)
    fr = [_host(a, rt) for a in (Mc, Rc, Mm, Rm)]
    cp = [_host(a, ct) for a in (Pc, Pm)]
    nout = T - int(N) + 1
    for a in fr + cp:
        if a.size != B * nout:
            raise ValueError(f"outputs must be [B, T-N+1] = [{B}, {nout}]")
    st = np.zeros((B, 8))
    rc = lib().oracle_sc_minn_check(x.ctypes.data, int(x.dtype == np.complex128), B, nb, T, int(N),
                                    fr[0].ctypes.data, cp[0].ctypes.data, fr[1].ctypes.data, fr[2].ctypes.data,
                                    cp[1].ctypes.data, fr[3].ctypes.data, int(f64), float(kP), float(kR), float(kM),
                                    st.ctypes.data, int(nthreads))
    if rc:
        raise RuntimeError(f"oracle_sc_minn_check failed ({rc})")
    return st


def zc_freq_check(x, N, cp, idx, tmpl, tmpl_energy, metric, eps, kM, nthreads=0):
    """Engine zc_freq metric [B, noff] (fp32 or fp64) against the direct-DFT fp64 reference of
    x [B, nb, T] (oracle_zc_freq_check).  Returns per-stream [B, 3]: max|dm|, max |dm|/bound,
    max oracle metric."""
    x = np.ascontiguousarray(x)
    if x.ndim == 2:
        x = x[:, None, :]
    if x.dtype not in (np.complex64, np.complex128):
        raise TypeError("x must be complex64 / complex128")
    B, nb, T = x.shape
    m = np.ascontiguousarray(metric)
    if m.dtype not in (np.float32, np.float64) or m.shape[0] != B or m.size != B * (T - N - cp + 1):
        raise ValueError("metric must be [B, T-N-cp+1] float32/float64")
    idx = np.ascontiguousarray(np.asarray(idx, np.int32))
    tb = np.ascontiguousarray(np.asarray(tmpl, np.complex128))
    st = np.zeros((B, 3))
    rc = lib().oracle_zc_freq_check(x.ctypes.data, int(x.dtype == np.complex128), B, nb, T, int(N), int(cp),
                                    int(idx.size), idx.ctypes.data, tb.ctypes.data, float(tmpl_energy),
                                    m.ctypes.data, int(m.dtype == np.float32), float(eps), float(kM),
                                    st.ctypes.data, int(nthreads))
    if rc:
        raise RuntimeError(f"oracle_zc_freq_check failed ({rc})")
    return st


def max_threads() -> int:
    return int(lib().oracle_max_threads())
