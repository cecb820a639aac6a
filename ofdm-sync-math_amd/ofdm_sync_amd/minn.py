"""Drop-in for the metrics of ``minn.py``.

minn_streaming_metric               (reference: minn.py:59-112; N from module global N_FFT)
minn_streaming_metric_parameterized (reference: minn.py:697-751)
"""
from __future__ import annotations

from ._metrics import window_metric

N_FFT = 2048  # core.py:6


def minn_streaming_metric(rx, *, precision=None):
    return window_metric("minn", rx, N_FFT, batched=False, precision=precision)


def minn_streaming_metric_parameterized(rx, symbol_len: int, *, precision=None):
    return window_metric("minn", rx, symbol_len, batched=False, precision=precision)


def minn_streaming_metric_batched(x, symbol_len: int | None = None, *, precision=None):
    return window_metric("minn", x, N_FFT if symbol_len is None else symbol_len, batched=True,
                         precision=precision)
