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


# ---- detector back end (combined_sc_min.py:167-259, :337-365), csrc/postproc.hip -------------
SMOOTH_WIN = 16          # combined_sc_min.py:265


def _trailing_average(x, win: int):
    """Trailing moving average (drop-in for combined_sc_min.py:167-180)."""
    from . import minn
    return minn._trailing_average(x, win)


def _streaming_peak_detector(metric, gate_mask):
    """First argmax over the first active gate run (drop-in for combined_sc_min.py:183-209);
    None if the gate never opens."""
    import numpy as np

    from . import _postproc
    metric = np.asarray(metric, dtype=float)
    gate_mask = np.asarray(gate_mask)
    if gate_mask.shape[0] != metric.shape[0]:
        raise ValueError("gate_mask must match metric length")
    if metric.size == 0:
        return None
    peak, st = _postproc.segment_peak_batched(metric, gate_mask.astype(bool))
    return None if int(st[0]) < 0 else int(peak[0])


def find_minn_peak(M, smooth_win: int = 8, gate_mask=None, search_bounds=None) -> int:
    """Minn timing inside the S&C gate (drop-in for combined_sc_min.py:212-259): trailing
    average of max(M, 0), then the streaming peak over the first run of gate_mask ∩ bounds."""
    import numpy as np

    from . import _postproc
    M = np.asarray(M, dtype=float)
    if M.size == 0:
        return 0
    if gate_mask is None:
        raise ValueError("Minn peak detection requires S&C gate mask")
    gate_mask = np.asarray(gate_mask)
    if gate_mask.shape[0] != M.shape[0]:
        raise ValueError("gate_mask must match metric length")
    Ms = _postproc.trailing_average(M, max(1, smooth_win), clip_negative=True)
    peak, st = _postproc.segment_peak_batched(Ms, gate_mask.astype(bool), search_bounds)
    if int(st[0]) < 0:
        raise ValueError("Minn peak detector received empty gate region")
    return int(peak[0])


def sc_gate_mask(M_sc, threshold: float = SC_GATE_THRESHOLD):
    """The S&C gate of run_simulation (combined_sc_min.py:337-358): (mask, (first, last + 1))."""
    from . import _postproc
    mask, span = _postproc.sc_gate_batched(M_sc, threshold)
    return _postproc.host_array(mask[0]), (int(span[0, 0]), int(span[0, 1]))


def detect_batched(M_minn, M_sc, *, smooth_win: int = SMOOTH_WIN, threshold: float = SC_GATE_THRESHOLD,
                   search_bounds=None):
    """The whole combined_sc_min decision on device metrics [B, n] (combined_sc_min.py:337-365):
    S&C gate -> trailing average of the Minn metric -> first-run peak.  Returns
    (peak [B] int64, status [B] int32, gate span [B, 2]); status -1 = empty gate region."""
    from . import _postproc
    mask, span = _postproc.sc_gate_batched(M_sc, threshold)
    Ms = _postproc.trailing_average(M_minn, max(1, smooth_win), clip_negative=True)
    peak, st = _postproc.segment_peak_batched(Ms, mask, search_bounds)
    return peak, st, span
