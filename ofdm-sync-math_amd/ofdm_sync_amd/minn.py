"""Drop-in for the metrics of ``minn.py``.

minn_streaming_metric               (reference: minn.py:59-112; N from module global N_FFT)
minn_streaming_metric_parameterized (reference: minn.py:697-751)
find_minn_peak / _trailing_average  (reference: minn.py:115-205; csrc/postproc.hip)
"""
from __future__ import annotations

import numpy as np

from ._metrics import window_metric

N_FFT = 2048  # core.py:6


def minn_streaming_metric(rx, *, precision=None):
    return window_metric("minn", rx, N_FFT, batched=False, precision=precision)


def minn_streaming_metric_parameterized(rx, symbol_len: int, *, precision=None):
    return window_metric("minn", rx, symbol_len, batched=False, precision=precision)


def minn_streaming_metric_batched(x, symbol_len: int | None = None, *, precision=None):
    return window_metric("minn", x, N_FFT if symbol_len is None else symbol_len, batched=True,
                         precision=precision)


def _trailing_average(x, win: int):
    """Trailing moving average (drop-in for minn.py:115-128), float64 recursion on the GPU."""
    from . import _postproc
    x = np.asarray(x, dtype=float)
    if x.size == 0:
        return x.copy()
    return _postproc.host_array(_postproc.trailing_average(x, win, clip_negative=False)[0])


def find_minn_peak(M, smooth_win: int = 8, gate_threshold: float = 0.5, search_bounds=None):
    """Timing from the Minn metric (drop-in for minn.py:131-205): (peak_idx, gate_mask, Ms).
    Gate = longest run of the trailing-average metric above gate_threshold * max; runs on
    ``ofs_trailing_average`` + ``ofs_minn_peak``.  Raises ValueError like the reference."""
    from . import _postproc
    M = np.asarray(M, dtype=float)
    if M.size == 0:
        raise ValueError("Minn metric is empty")
    peak, glo, ghi, Ms, st = _postproc.minn_peak_batched(M, smooth_win, gate_threshold, search_bounds)
    status = int(st[0])
    if status == -2:
        raise ValueError("Minn metric did not produce a positive peak")
    if status < 0:
        raise ValueError("Minn metric is empty")
    gate = np.zeros(M.size, dtype=bool)
    gate[int(glo[0]):int(ghi[0])] = True
    return int(peak[0]), gate, _postproc.host_array(Ms[0])


def find_minn_peak_batched(M, smooth_win: int = 8, gate_threshold: float = 0.5, search_bounds=None):
    """Batched find_minn_peak over M[B, n] (device tensors): (peak, gate_lo, gate_hi, Ms, status);
    gate of stream b = [gate_lo[b], gate_hi[b]); status < 0 where the reference raises."""
    from . import _postproc
    return _postproc.minn_peak_batched(M, smooth_win, gate_threshold, search_bounds)
