"""Drop-in for ``sc.sc_streaming_metric`` (reference: sc.py:42-78).

Like the reference, the symbol length is read from the module global ``N_FFT`` at call time
(override ``sc.N_FFT`` to re-parameterise).  Computed by ``ofs_sc_metric`` (r_mode 0).
"""
from __future__ import annotations

from ._metrics import window_metric

N_FFT = 2048            # core.py:6
CYCLIC_PREFIX = 512     # core.py:8


def sc_streaming_metric(rx, *, precision=None):
    """Schmidl & Cox streaming metric: returns (M, P_sum, R_sum) of length T - N_FFT + 1."""
    return window_metric("sc", rx, N_FFT, batched=False, precision=precision)


def sc_streaming_metric_batched(x, N: int | None = None, *, precision=None):
    """Batched S&C metric over x[B, n_branch, T]; device tensors [B, T-N+1]."""
    return window_metric("sc", x, N_FFT if N is None else N, batched=True, precision=precision)
