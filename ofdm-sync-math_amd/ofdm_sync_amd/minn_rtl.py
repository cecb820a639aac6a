"""Drop-in for the RTL-style Minn metric of ``minn_rtl.py``.

minn_rtl_streaming_metric (reference: minn_rtl.py:667-733) -> MinnRTLMetricState
detect_minn_rtl           (reference: minn_rtl.py:750-825) -> MinnRTLDetection

The correlation/energy pipeline of ``_antenna_path`` (minn_rtl.py:583-652) runs on the HIP
window-metric engine in fp64: on integer (ADC) inputs every value equals the reference's
float64 integers exactly.  The IIR smoothing is inherently sequential per stream and is
run as the reference's exact float64 recursion (one wave per stream), fused with the
threshold compare and, for the batched API, the gate FSM.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

N_FFT = 2048                                   # core.py:6
SMOOTH_SHIFT = 3                               # minn_rtl.py:831
THRESH_FRAC_BITS = 15                          # minn_rtl.py:832
THRESH_VALUE = int(0.10 * (1 << THRESH_FRAC_BITS))
HYSTERESIS = 2
PREAMBLE_Q = N_FFT // 4
TIMING_OFFSET = 0

_SMOOTH_MODES = {"float": 0, "floor": 1}


@dataclass
class MinnRTLMetricState:
    corr_total: np.ndarray
    corr_positive: np.ndarray
    smooth_metric: np.ndarray
    energy_total: np.ndarray
    corr_scaled: np.ndarray
    energy_scaled: np.ndarray
    metric_valid: np.ndarray
    above_threshold: np.ndarray


@dataclass
class MinnRTLEvent:
    peak_index: int
    detected_index: int
    gate_segment: tuple[int, int]


@dataclass
class MinnRTLDetection:
    events: list[MinnRTLEvent]
    gate_mask: np.ndarray
    gate_segments: list[tuple[int, int]]


@dataclass
class MinnRTLBatch:
    """Device-resident batched result: every array [B, T]; events [B, E, 4] =
    (peak_index, detected_index, seg_start, seg_end); open_gate_start [B] (-1: none)."""
    corr_total: torch.Tensor
    corr_positive: torch.Tensor
    smooth_metric: torch.Tensor
    energy_total: torch.Tensor
    corr_scaled: torch.Tensor
    energy_scaled: torch.Tensor
    metric_valid: torch.Tensor
    above_threshold: torch.Tensor
    n_events: torch.Tensor | None = None
    events: torch.Tensor | None = None
    open_gate_start: torch.Tensor | None = None


def _run(batch, Q, smooth_shift, threshold_value, threshold_frac_bits, smooth_mode, detect,
         hysteresis, timing_offset, max_events):
    dev = batch.data.device
    B, T = batch.B, batch.T
    f = lambda: torch.empty((B, T), dtype=torch.float64, device=dev)  # noqa: E731
    b = lambda: torch.empty((B, T), dtype=torch.bool, device=dev)     # noqa: E731
    out = MinnRTLBatch(f(), f(), f(), f(), f(), f(), b(), b())
    if detect:
        out.n_events = torch.zeros((B,), dtype=torch.int32, device=dev)
        out.events = torch.empty((B, max(max_events, 1), 4), dtype=torch.int64, device=dev)
        out.open_gate_start = torch.empty((B,), dtype=torch.int64, device=dev)
    rc = _lib.lib().ofs_minn_rtl(
        batch.fmt, batch.data.data_ptr(), B, batch.nb, T, int(Q), int(smooth_shift),
        _SMOOTH_MODES[smooth_mode], int(threshold_value), int(threshold_frac_bits),
        out.corr_total.data_ptr(), out.corr_positive.data_ptr(), out.smooth_metric.data_ptr(),
        out.energy_total.data_ptr(), out.corr_scaled.data_ptr(), out.energy_scaled.data_ptr(),
        out.metric_valid.data_ptr(), out.above_threshold.data_ptr(), int(detect), int(hysteresis),
        int(timing_offset), int(max_events), _lib.ptr(out.n_events), _lib.ptr(out.events),
        _lib.ptr(out.open_gate_start), _lib.stream_ptr())
    _lib.check(rc, "ofs_minn_rtl")
    return out


def minn_rtl_batched(x, quarter_len: int, *, smooth_shift: int = SMOOTH_SHIFT,
                     threshold_value: int = THRESH_VALUE, threshold_frac_bits: int = THRESH_FRAC_BITS,
                     smooth_mode: str = "float", detect: bool = True, hysteresis: int = HYSTERESIS,
                     timing_offset: int = TIMING_OFFSET, max_events: int = 16) -> MinnRTLBatch:
    """Batched RTL metric + gate over x[B, n_branch, T] (complex or int16 I/Q [..., 2])."""
    if quarter_len <= 0:
        raise ValueError("quarter_len must be positive.")
    batch = _lib.as_batch(x, batched=True, complex_cast=True)
    out = _run(batch, quarter_len, smooth_shift, threshold_value, threshold_frac_bits, smooth_mode,
               detect, hysteresis, timing_offset, max_events)
    if detect and batch.B > 0 and batch.T > 0:
        worst = int(out.n_events.max().item())
        if worst > max_events:
            out = _run(batch, quarter_len, smooth_shift, threshold_value, threshold_frac_bits,
                       smooth_mode, detect, hysteresis, timing_offset, worst)
    return out


def minn_rtl_streaming_metric(
    rx,
    *,
    smooth_shift: int,
    threshold_value: int,
    threshold_frac_bits: int,
    quarter_len: int | None = None,
    smooth_mode: str = "float",
) -> MinnRTLMetricState:
    """RTL-aligned Minn timing metric across all branches (drop-in for minn_rtl.py:667-733)."""
    batch = _lib.as_batch(rx, batched=False, complex_cast=True)
    if quarter_len is None:
        quarter_len = N_FFT // 4
    if quarter_len <= 0:
        raise ValueError("quarter_len must be positive.")
    out = _run(batch, quarter_len, smooth_shift, threshold_value, threshold_frac_bits, smooth_mode,
               False, 0, 0, 0)
    names = ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled",
             "energy_scaled", "metric_valid", "above_threshold")
    vals = {k: getattr(out, k)[0] for k in names}
    if batch.from_numpy:
        vals = {k: _lib.to_host(v) for k, v in vals.items()}
    return MinnRTLMetricState(**vals)


def detect_minn_rtl(state: MinnRTLMetricState, *, hysteresis: int, timing_offset: int) -> MinnRTLDetection:
    """Gate and peak tracking of the RTL detector (drop-in for minn_rtl.py:750-825)."""
    dev = _lib.require_gpu()

    def dt(a, dtype):
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
        return t.to(device=dev, dtype=dtype).contiguous()

    cp = dt(state.corr_positive, torch.float64)
    ab = dt(state.above_threshold, torch.uint8)
    vd = dt(state.metric_valid, torch.uint8)
    T = int(cp.numel())
    segments: list[tuple[int, int]] = []
    events: list[MinnRTLEvent] = []
    if T > 0:
        max_ev = 16
        while True:
            n_ev = torch.zeros((1,), dtype=torch.int32, device=dev)
            ev = torch.empty((1, max_ev, 4), dtype=torch.int64, device=dev)
            op = torch.empty((1,), dtype=torch.int64, device=dev)
            rc = _lib.lib().ofs_minn_rtl_gate(cp.data_ptr(), ab.data_ptr(), vd.data_ptr(), 1, T,
                                              int(hysteresis), int(timing_offset), max_ev,
                                              n_ev.data_ptr(), ev.data_ptr(), op.data_ptr(),
                                              _lib.stream_ptr())
            _lib.check(rc, "ofs_minn_rtl_gate")
            n = int(n_ev.item())
            if n <= max_ev:
                break
            max_ev = n
        evh = ev[0, :n].cpu().numpy()
        for r in evh:
            seg = (int(r[2]), int(r[3]))
            segments.append(seg)
            events.append(MinnRTLEvent(peak_index=int(r[0]), detected_index=int(r[1]), gate_segment=seg))
        o = int(op.item())
        if o >= 0:
            segments.append((o, T))
    gate_mask = np.zeros(T, dtype=bool)
    for a, b in segments:
        gate_mask[a:b] = True
    return MinnRTLDetection(events=events, gate_mask=gate_mask, gate_segments=segments)
