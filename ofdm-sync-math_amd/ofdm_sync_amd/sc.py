"""Drop-in for ``sc.sc_streaming_metric`` (reference: sc.py:42-78).

Like the reference, the symbol length is read from the module global ``N_FFT`` at call time
(override ``sc.N_FFT`` to re-parameterise).  Computed by ``ofs_sc_metric`` (r_mode 0).
``find_plateau_end_from_metric`` (sc.py:81-146) runs on ``ofs_plateau_end``.
"""
from __future__ import annotations

import numpy as np

from ._metrics import window_metric

N_FFT = 2048            # core.py:6
CYCLIC_PREFIX = 512     # core.py:8


def sc_streaming_metric(rx, *, precision=None):
    """Schmidl & Cox streaming metric: returns (M, P_sum, R_sum) of length T - N_FFT + 1."""
    return window_metric("sc", rx, N_FFT, batched=False, precision=precision)


def sc_streaming_metric_batched(x, N: int | None = None, *, precision=None):
    """Batched S&C metric over x[B, n_branch, T]; device tensors [B, T-N+1]."""
    return window_metric("sc", x, N_FFT if N is None else N, batched=True, precision=precision)


def find_plateau_end_from_metric(M, cp_len: int, lookahead: int | None = None, smooth_win: int = 8) -> int:
    """End of the first S&C plateau (drop-in for sc.py:81-146), computed by ``ofs_plateau_end``."""
    from . import _postproc
    M = np.asarray(M) if not hasattr(M, "dim") else M
    if (M.size if isinstance(M, np.ndarray) else M.numel()) == 0:
        return 0
    idx, _, st = _postproc.plateau_end_batched(M, cp_len, lookahead=lookahead, smooth_win=smooth_win)
    if int(st[0]) == -3:
        raise ValueError("operands could not be broadcast together (sc.py:141)")
    return int(idx[0])


def find_plateau_end_batched(M, cp_len: int, lookahead: int | None = None, smooth_win: int = 8):
    """Batched plateau end over M[B, n]: (index [B] int64, smoothed metric, branch status [B])."""
    from . import _postproc
    return _postproc.plateau_end_batched(M, cp_len, lookahead=lookahead, smooth_win=smooth_win)
