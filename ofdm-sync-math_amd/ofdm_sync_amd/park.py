"""Drop-in for ``park.park_streaming_metric`` (reference: park.py:64-114).

Like the reference, the symbol length is read from the module global ``N_FFT`` at call time.
Computed by ``ofs_park_metric`` (csrc/corr.hip): an LDS-staged direct mirror product, fp64
for complex128 / integer inputs, fp32 for complex64 tensors unless ``precision`` says otherwise.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

N_FFT = 2048            # core.py:6


def _run(batch: _lib.Batch, N: int, prec: int):
    dev = batch.data.device
    half = N // 2
    nout = batch.T - 2 * half if (half > 0 and batch.T >= 2 * half + 1) else 0
    M = _lib.out_real((batch.B, nout), prec, dev)
    P = _lib.out_cplx((batch.B, nout), prec, dev)
    E = _lib.out_real((batch.B, nout), prec, dev)
    if nout > 0:
        rc = _lib.lib().ofs_park_metric(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T,
                                        int(N), prec, M.data_ptr(), P.data_ptr(), E.data_ptr(),
                                        _lib.stream_ptr())
        _lib.check(rc, "ofs_park_metric")
    ds = torch.arange(half, half + nout, dtype=torch.int64, device=dev)
    return ds, M, P, E


def park_streaming_metric(rx, *, precision=None):
    """Park timing metric across receive branches: returns (ds, M, P_sum, E_sum)."""
    batch = _lib.as_batch(rx, batched=False)
    prec = _lib.resolve_precision(batch, precision)
    ds, M, P, E = _run(batch, int(N_FFT), prec)
    if batch.from_numpy:
        return (_lib.to_host(ds), _lib.to_host(M[0], np.float64), _lib.to_host(P[0], np.complex128),
                _lib.to_host(E[0], np.float64))
    return ds, M[0], P[0], E[0]


def park_streaming_metric_batched(x, N: int | None = None, *, precision=None):
    """Batched Park metric over x[B, n_branch, T]: (ds, M, P, E), device tensors [B, T-2*(N//2)]."""
    batch = _lib.as_batch(x, batched=True)
    prec = _lib.resolve_precision(batch, precision)
    return _run(batch, int(N_FFT if N is None else N), prec)
