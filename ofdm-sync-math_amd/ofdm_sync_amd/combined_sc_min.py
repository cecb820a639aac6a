"""Drop-in for the metrics of ``combined_sc_min.py``.

minn_streaming_metric        (reference: combined_sc_min.py:60-113; Q = N_FFT//4, module global)
schmidl_cox_streaming_metric (reference: combined_sc_min.py:116-164; R = both halves)
Both run on the HIP window-metric engine (``ofs_minn_metric`` / ``ofs_sc_metric`` r_mode 1).
"""
from __future__ import annotations

from ._metrics import window_metric

N_FFT = 2048            # core.py:6
SC_GATE_THRESHOLD = 0.6  # combined_sc_min.py:267


def minn_streaming_metric(rx, *, precision=None):
    """Minn metric with 4-part correlation; returns (M, P_sum, R_sum)."""
    return window_metric("minn", rx, N_FFT, batched=False, precision=precision)


def schmidl_cox_streaming_metric(rx, symbol_len: int = N_FFT, *, precision=None):
    """S&C metric for a symbol with two identical halves; returns (M_sc, P_sum, R_sum)."""
    return window_metric("comb", rx, symbol_len, batched=False, precision=precision)


def schmidl_cox_streaming_metric_batched(x, symbol_len: int = N_FFT, *, precision=None):
    return window_metric("comb", x, symbol_len, batched=True, precision=precision)


def minn_streaming_metric_batched(x, symbol_len: int | None = None, *, precision=None):
    return window_metric("minn", x, N_FFT if symbol_len is None else symbol_len, batched=True,
                         precision=precision)


def sc_minn_streaming_metrics_batched(x, symbol_len: int | None = None, *, precision=None):
    """Both detector metrics of combined_sc_min.run_simulation (combined_sc_min.py:333-334) in
    one pass: ((M_minn, P_minn, R_minn), (M_sc, P_sc, R_sc)), device tensors [B, T-N+1].
    Runs the fused kernel (``ofs_sc_minn_metric``) where it applies."""
    import torch

    from . import _lib
    N = int(N_FFT if symbol_len is None else symbol_len)
    batch = _lib.as_batch(x, batched=True)
    prec = _lib.resolve_precision(batch, precision)
    dev = batch.data.device
    if N % 2:
        raise ValueError(f"operands could not be broadcast together: odd symbol length {N}")
    n_out = max(batch.T - N + 1, 0)
    outs = [_lib.out_real((batch.B, n_out), prec, dev), _lib.out_cplx((batch.B, n_out), prec, dev),
            _lib.out_real((batch.B, n_out), prec, dev), _lib.out_real((batch.B, n_out), prec, dev),
            _lib.out_cplx((batch.B, n_out), prec, dev), _lib.out_real((batch.B, n_out), prec, dev)]
    if n_out > 0 and batch.B > 0:
        rc = _lib.lib().ofs_sc_minn_metric(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T, N,
                                           prec, *[t.data_ptr() for t in outs], _lib.stream_ptr())
        _lib.check(rc, "ofs_sc_minn_metric")
    del torch
    return (outs[3], outs[4], outs[5]), (outs[0], outs[1], outs[2])
