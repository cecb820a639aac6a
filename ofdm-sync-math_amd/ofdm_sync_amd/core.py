"""Drop-in for the CP-correlation CFO estimators of ``core.py`` (reference: core.py:179-336):
estimate_cfo_from_cp, estimate_cfo_from_cp_robust, estimate_cfo_from_cp_peak[_with_index],
find_cp_start_via_corr.

Only these hot-path functions are mirrored; the builders, plotting and receiver back-end of the
reference's core.py are out of scope.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

N_FFT = 2048
NUM_ACTIVE_SUBCARRIERS = 1200
CYCLIC_PREFIX = 512
TX_PRE_PAD_SAMPLES = 1337
SAMPLE_RATE_HZ = 30_720_000.0


def estimate_cfo_from_cp_batched(x, starts, n_fft: int, cp_len: int, fs_hz: float, *, return_P=False):
    """CFO (Hz) per stream of x[B, n_branch, T] from the CP at starts[B] (device tensors)."""
    batch = _lib.as_batch(x, batched=True)
    dev = batch.data.device
    st = starts if isinstance(starts, torch.Tensor) else torch.as_tensor(np.asarray(starts))
    st = st.to(device=dev, dtype=torch.int64).contiguous()
    if st.numel() != batch.B:
        raise ValueError("starts must have one entry per stream")
    if batch.B and (int(st.min()) < 0 or int(st.max()) + n_fft + cp_len > batch.T):
        raise ValueError("CP windows must lie inside the stream")
    cfo = torch.empty((batch.B,), dtype=torch.float64, device=dev)
    P = torch.empty((batch.B, 2), dtype=torch.float64, device=dev)
    rc = _lib.lib().ofs_cp_cfo(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T,
                               st.data_ptr(), int(n_fft), int(cp_len), float(fs_hz), P.data_ptr(),
                               cfo.data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "ofs_cp_cfo")
    return (cfo, torch.view_as_complex(P)) if return_P else cfo


def estimate_cfo_from_cp(rx, start: int, n_fft: int, cp_len: int, fs_hz: float) -> float:
    """Estimate CFO (Hz) from CP correlation on a symbol whose CP starts at `start`."""
    a = rx if isinstance(rx, torch.Tensor) else np.asarray(rx)
    T = a.shape[-1]
    start, n_fft, cp_len = int(start), int(n_fft), int(cp_len)
    if start < 0 or n_fft < 0 or cp_len < 0:
        raise ValueError("start, n_fft and cp_len must be non-negative")
    la = max(0, min(cp_len, T - start))
    lb = max(0, min(cp_len, T - start - n_fft))
    if la != lb:
        # numpy would fail to broadcast the truncated slices (core.py:190-192)
        raise ValueError(f"operands could not be broadcast together with shapes ({la},) ({lb},)")
    if la == 0:
        return float(-np.angle(0j) * fs_hz / (2 * np.pi * n_fft))
    x = a[None] if a.ndim == 1 else a
    cfo = estimate_cfo_from_cp_batched(x[None], [start], n_fft, la, fs_hz)
    return float(cfo[0].item())


# ---------------------------------------------------------------------------------------------
# CP-correlation searches around an estimated start (core.py:199-336) -> ofs_cp_search
# ---------------------------------------------------------------------------------------------
CPS_ROBUST, CPS_PEAK = 0, 1


def cp_search_batched(x, est, n_fft: int, win_len: int, span: int, mode: int, fs_hz: float):
    """One CP search per stream of x[B, n_branch, T] around est[B] (device-resident result).

    mode CPS_ROBUST: cfo from the angle of sum_d P_win(d) (estimate_cfo_from_cp_robust);
    mode CPS_PEAK: d* = first argmax |P_win(d)|, cfo from P_win(d*) (estimate_cfo_from_cp_peak,
    find_cp_start_via_corr).  Returns (cfo [B] f64, d [B] int64, P [B] c128, status [B] int32);
    status 1 = empty search range (the reference falls back to estimate_cfo_from_cp at est)."""
    batch = _lib.as_batch(x, batched=True)
    dev = batch.data.device
    e = est if isinstance(est, torch.Tensor) else torch.as_tensor(np.asarray(est))
    e = e.to(device=dev, dtype=torch.int64).contiguous()
    if e.numel() != batch.B:
        raise ValueError("est must have one entry per stream")
    cfo = torch.empty((batch.B,), dtype=torch.float64, device=dev)
    d = torch.empty((batch.B,), dtype=torch.int64, device=dev)
    P = torch.empty((batch.B, 2), dtype=torch.float64, device=dev)
    st = torch.empty((batch.B,), dtype=torch.int32, device=dev)
    rc = _lib.lib().ofs_cp_search(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T, e.data_ptr(),
                                  int(n_fft), int(win_len), int(span), int(mode), float(fs_hz), P.data_ptr(),
                                  d.data_ptr(), cfo.data_ptr(), st.data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "ofs_cp_search")
    return cfo, d, torch.view_as_complex(P), st


def _search_one(rx, est, n_fft, win, span, mode, fs_hz):
    a = rx if isinstance(rx, torch.Tensor) else np.asarray(rx)
    x = a[None] if a.ndim == 1 else a
    cfo, d, _, st = cp_search_batched(x[None], [int(est)], n_fft, win, span, mode, fs_hz)
    return float(cfo[0].item()), int(d[0].item()), int(st[0].item()), x


def estimate_cfo_from_cp_robust(rx, cp_start_est: int, n_fft: int, cp_len: int, fs_hz: float,
                                span: int | None = None, win_len: int | None = None) -> float:
    """Robust CFO estimate by aggregating CP correlations around an estimated start."""
    span = cp_len // 2 if span is None else int(max(0, span))
    win = cp_len // 2 if win_len is None else int(max(1, win_len))
    if win < 1:                                        # cp_len < 2: every window is empty
        a = np.asarray(rx) if not isinstance(rx, torch.Tensor) else rx
        T = a.shape[-1]
        if min(T - n_fft, cp_start_est + span) > max(0, cp_start_est - span):
            return float(-np.angle(0j) * fs_hz / (2 * np.pi * n_fft))
        return estimate_cfo_from_cp(rx, cp_start_est, n_fft, 0, fs_hz)
    cfo, _, st, x = _search_one(rx, cp_start_est, n_fft, win, span, CPS_ROBUST, fs_hz)
    if st == 1:                                        # core.py:222-223
        return estimate_cfo_from_cp(x, cp_start_est, n_fft, min(cp_len, win), fs_hz)
    return cfo


def estimate_cfo_from_cp_peak_with_index(rx, cp_start_est: int, n_fft: int, cp_len: int, fs_hz: float,
                                         span: int | None = None) -> tuple[float, int]:
    """Like estimate_cfo_from_cp_peak, but also return the best CP offset index used."""
    span = cp_len // 2 if span is None else int(max(0, span))
    if cp_len < 1:
        raise ValueError("cp_len must be positive")
    cfo, d, st, x = _search_one(rx, cp_start_est, n_fft, cp_len, span, CPS_PEAK, fs_hz)
    if st == 1:                                        # core.py:287-288
        return estimate_cfo_from_cp(x, cp_start_est, n_fft, cp_len, fs_hz), int(cp_start_est)
    return cfo, d


def estimate_cfo_from_cp_peak(rx, cp_start_est: int, n_fft: int, cp_len: int, fs_hz: float,
                              span: int | None = None) -> float:
    """Pick the CP offset with maximum |P(d)| near the estimated CP start and use its phase."""
    return estimate_cfo_from_cp_peak_with_index(rx, cp_start_est, n_fft, cp_len, fs_hz, span)[0]


def find_cp_start_via_corr(rx, est_start: int, n_fft: int, cp_len: int, search_half: int = 1024) -> int:
    """Refine CP start using the magnitude of CP correlation |P(d)| (core.py:306-336)."""
    if cp_len < 1:
        raise ValueError("cp_len must be positive")
    _, d, _, _ = _search_one(rx, est_start, n_fft, cp_len, max(0, int(search_half)), CPS_PEAK, 0.0)
    return d
