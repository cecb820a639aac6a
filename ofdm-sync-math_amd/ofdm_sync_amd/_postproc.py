"""Detection post-processing on the GPU (csrc/postproc.hip): metric streams -> timing decisions.

Batched device-resident entry points, shared by the drop-in functions of ``sc``, ``minn`` and
``combined_sc_min``:

  trailing_average      minn._trailing_average (minn.py:115-128)
  plateau_end_batched   sc.find_plateau_end_from_metric (sc.py:81-146)
  minn_peak_batched     minn.find_minn_peak (minn.py:131-205)
  sc_gate_batched       S&C gate of combined_sc_min.run_simulation (combined_sc_min.py:337-358)
  segment_peak_batched  combined_sc_min._streaming_peak_detector (combined_sc_min.py:183-209)

Metrics are [B, n] tensors (f32 or f64, any device: moved to the GPU); results stay on the GPU.
A 1-D metric is one stream.  No CPU fallback: the HIP library and a GPU are required.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

# ofs_plateau_end status codes (include/ofdmsync.h)
PLATEAU_BRANCH = {0: "empty", 1: "drop95", 2: "run60", 3: "slope", 4: "slope_empty"}


def _metric(M) -> tuple[torch.Tensor, int, bool]:
    """[B, n] contiguous device tensor of a real metric, its ABI precision, and whether it came
    from numpy (drop-in callers get numpy back)."""
    dev = _lib.require_gpu()
    from_numpy = not isinstance(M, torch.Tensor)
    t = torch.from_numpy(np.ascontiguousarray(np.asarray(M, dtype=np.float64))) if from_numpy else M
    if t.is_complex():
        raise TypeError("metric must be real")
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    if t.device.type != "cuda":
        t = t.to(dev)
    if t.dim() == 1:
        t = t[None]
    if t.dim() != 2:
        raise ValueError("metric must be [n] or [B, n]")
    t = t.contiguous()
    return t, (_lib.FP64 if t.dtype == torch.float64 else _lib.FP32), from_numpy


def bounds(n: int, search_bounds) -> tuple[int, int]:
    """search_bounds clipped like the reference (minn.py:186-193): None or start >= end -> all."""
    if search_bounds is None:
        return 0, n
    start, end = max(0, int(search_bounds[0])), min(n, int(search_bounds[1]))
    return (0, n) if start >= end else (start, end)


def trailing_average(x, win: int, clip_negative: bool = True) -> torch.Tensor:
    """Trailing moving average [B, n] f64 of max(x, 0) (clip_negative) or x."""
    t, prec, _ = _metric(x)
    B, n = t.shape
    out = torch.empty((B, n), dtype=torch.float64, device=t.device)
    rc = _lib.lib().ofs_trailing_average(prec, t.data_ptr(), B, n, int(win), int(bool(clip_negative)),
                                         out.data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "ofs_trailing_average")
    return out


def plateau_end_batched(M, cp_len: int, lookahead: int | None = None, smooth_win: int = 8):
    """Per-stream sc.find_plateau_end_from_metric: (index [B] int64, Ms [B, max(n, w)] f64,
    status [B] int32 = branch taken, -3 where numpy would raise on a broadcast)."""
    t, prec, _ = _metric(M)
    B, n = t.shape
    w = max(1, int(smooth_win))
    Ms = torch.empty((B, max(n, w)), dtype=torch.float64, device=t.device)
    idx = torch.empty((B,), dtype=torch.int64, device=t.device)
    st = torch.empty((B,), dtype=torch.int32, device=t.device)
    rc = _lib.lib().ofs_plateau_end(prec, t.data_ptr(), B, n, int(cp_len), -1 if lookahead is None else int(lookahead),
                                    w, Ms.data_ptr(), idx.data_ptr(), st.data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "ofs_plateau_end")
    return idx, Ms, st


def minn_peak_batched(M, smooth_win: int = 8, gate_threshold: float = 0.5, search_bounds=None):
    """Per-stream minn.find_minn_peak: (peak [B], gate_lo [B], gate_hi [B], Ms [B, n], status [B]);
    the gate of stream b is [gate_lo, gate_hi); status -1 empty metric, -2 no positive peak."""
    t, _, _ = _metric(M)
    B, n = t.shape
    Ms = trailing_average(t, max(1, int(smooth_win)), True)
    lo, hi = bounds(n, search_bounds)
    peak, glo, ghi = (torch.empty((B,), dtype=torch.int64, device=t.device) for _ in range(3))
    st = torch.empty((B,), dtype=torch.int32, device=t.device)
    rc = _lib.lib().ofs_minn_peak(Ms.data_ptr(), B, n, float(gate_threshold), lo, hi, peak.data_ptr(),
                                  glo.data_ptr(), ghi.data_ptr(), st.data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "ofs_minn_peak")
    return peak, glo, ghi, Ms, st


def sc_gate_batched(M_sc, threshold: float = 0.6):
    """S&C gate per stream: (mask [B, n] bool, span [B, 2] int64 = first, last + 1)."""
    t, prec, _ = _metric(M_sc)
    B, n = t.shape
    if n == 0:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    mask = torch.empty((B, n), dtype=torch.bool, device=t.device)
    span = torch.empty((B, 2), dtype=torch.int64, device=t.device)
    rc = _lib.lib().ofs_sc_gate(prec, t.data_ptr(), B, n, float(threshold), mask.data_ptr(), span.data_ptr(),
                                _lib.stream_ptr())
    _lib.check(rc, "ofs_sc_gate")
    return mask, span


def segment_peak_batched(Ms, mask, search_bounds=None):
    """First argmax (strict >) of Ms over the first run of mask within the bounds, per stream:
    (peak [B] int64, status [B] int32; -1 = empty gate region)."""
    t, _, _ = _metric(Ms)
    if t.dtype != torch.float64:
        t = t.to(torch.float64)
    B, n = t.shape
    m = mask if isinstance(mask, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(mask, bool)))
    m = m.to(device=t.device, dtype=torch.bool)
    if m.dim() == 1:
        m = m[None]
    if tuple(m.shape) != (B, n):
        raise ValueError("gate_mask must match metric length")
    m = m.contiguous()
    lo, hi = bounds(n, search_bounds)
    peak = torch.empty((B,), dtype=torch.int64, device=t.device)
    st = torch.empty((B,), dtype=torch.int32, device=t.device)
    rc = _lib.lib().ofs_segment_peak(t.data_ptr(), m.data_ptr(), B, n, lo, hi, peak.data_ptr(), st.data_ptr(),
                                     _lib.stream_ptr())
    _lib.check(rc, "ofs_segment_peak")
    return peak, st


def host_array(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()
