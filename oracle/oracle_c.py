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


def max_threads() -> int:
    return int(lib().oracle_max_threads())
