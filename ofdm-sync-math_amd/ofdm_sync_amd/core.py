"""Drop-in for the CP-correlation CFO estimator of ``core.py`` (reference: core.py:179-196).

Only the hot-path function is mirrored; the builders, plotting and receiver back-end of the
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
