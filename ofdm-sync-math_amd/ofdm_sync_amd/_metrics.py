"""Shared host wrappers for the sliding-window metrics (S&C / combined S&C / Minn)."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

_SC, _COMB, _MINN = "sc", "comb", "minn"


def _empty(from_numpy: bool, dev):
    if from_numpy:
        return np.zeros(0), np.zeros(0, dtype=complex), np.zeros(0)
    return (torch.zeros(0, dtype=torch.float64, device=dev),
            torch.zeros(0, dtype=torch.complex128, device=dev),
            torch.zeros(0, dtype=torch.float64, device=dev))


def window_metric(kind: str, x, N: int, *, batched: bool, precision=None):
    """Run one of the S&C/Minn window metrics.  Returns (M, P, R).

    Unbatched: 1-D/2-D reference inputs -> numpy (or torch) arrays of length T-N+1.
    Batched: [B, n_branch, T] -> device tensors [B, T-N+1].
    """
    batch = _lib.as_batch(x, batched=batched)
    prec = _lib.resolve_precision(batch, precision)
    dev = batch.data.device
    N = int(N)
    n_out = batch.T - N + 1
    if kind in (_SC, _COMB):
        if N // 2 == 0 or n_out <= 0:
            if batched:
                return (_lib.out_real((batch.B, 0), prec, dev), _lib.out_cplx((batch.B, 0), prec, dev),
                        _lib.out_real((batch.B, 0), prec, dev))
            return _empty(batch.from_numpy, dev)
        if N % 2:
            # the reference slices x[0:half] against x[half:N] (N-half elements): broadcasting
            # fails for odd N (sc.py:60, combined_sc_min.py:150-151)
            raise ValueError(f"operands could not be broadcast together: odd symbol length {N}")
    else:
        if n_out <= 0:
            if batched:
                return (_lib.out_real((batch.B, 0), prec, dev), _lib.out_cplx((batch.B, 0), prec, dev),
                        _lib.out_real((batch.B, 0), prec, dev))
            return _empty(batch.from_numpy, dev)
    M = _lib.out_real((batch.B, n_out), prec, dev)
    P = _lib.out_cplx((batch.B, n_out), prec, dev)
    R = _lib.out_real((batch.B, n_out), prec, dev)
    L = _lib.lib()
    if kind == _MINN:
        rc = L.ofs_minn_metric(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T, N, prec,
                               M.data_ptr(), P.data_ptr(), R.data_ptr(), _lib.stream_ptr())
        _lib.check(rc, "ofs_minn_metric")
    else:
        rc = L.ofs_sc_metric(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T, N,
                             1 if kind == _COMB else 0, prec, M.data_ptr(), P.data_ptr(), R.data_ptr(),
                             _lib.stream_ptr())
        _lib.check(rc, "ofs_sc_metric")
    if batched:
        return M, P, R
    if batch.from_numpy:
        return (_lib.to_host(M[0], np.float64), _lib.to_host(P[0], np.complex128),
                _lib.to_host(R[0], np.float64))
    return M[0], P[0], R[0]
