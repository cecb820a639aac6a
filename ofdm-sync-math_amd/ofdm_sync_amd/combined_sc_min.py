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
