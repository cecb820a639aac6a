"""Drop-in for the [A][A] streaming detector of ``sync_aa.py`` (reference: sync_aa.py:421-571).

``aa_detect_streaming`` keeps the reference signature, defaults, dataclasses and field
names; the P/R/M streams and the gate/peak/CFO events are computed by one fused HIP kernel
(``ofs_aa_detect``).  ``aa_detect_streaming_batched`` is the native fast path: a batch of
independent receive streams [B, n_ant, T], device-resident in and out.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

# System constants (sync_aa.py:99-125)
N_FFT = 1024
NUM_ACTIVE_SUBCARRIERS = 600
CYCLIC_PREFIX = 72
SAMPLE_RATE_HZ = 15_360_000.0
PREAMBLE_LENGTHS = [1024, 512, 256]
DEFAULT_PREAMBLE_LEN = 1024
PREAMBLE_HALF_LEN = DEFAULT_PREAMBLE_LEN // 2
PREAMBLE_TOTAL_LEN = DEFAULT_PREAMBLE_LEN
DETECT_THRESHOLD = 0.15
DETECT_HYSTERESIS = 128
ADC_BITS = 12
ADC_LEVELS = 2 ** (ADC_BITS - 1)
TX_PRE_PAD_SAMPLES = 500
TX_POST_PAD_SAMPLES = 500


@dataclass
class AADetectorState:
    """State arrays from streaming detection (sync_aa.py:392-398)."""
    P: np.ndarray
    R: np.ndarray
    M: np.ndarray
    valid: np.ndarray


@dataclass
class AADetectionEvent:
    """A single detection event (sync_aa.py:401-410)."""
    peak_index: int
    P_at_peak: complex
    M_at_peak: float
    gate_start: int
    gate_end: int
    cfo_hz: float
    frame_start: int


@dataclass
class AADetectionResult:
    """Complete detection result (sync_aa.py:413-418)."""
    events: list[AADetectionEvent]
    state: AADetectorState
    num_antennas: int


@dataclass
class AABatchResult:
    """Device-resident result of ``aa_detect_streaming_batched``.

    P [B,T] complex, R/M [B,T] real, valid [B,T] bool (None when not requested);
    n_events [B] int32; ev_int [B,E,4] int64 = (peak_index, gate_start, gate_end, frame_start);
    ev_real [B,E,4] f64 = (P_re, P_im, M_at_peak, cfo_hz); E = max_events.  Only the first
    min(n_events[b], E) slots of stream b are written; the rest are undefined (the buffers are
    not cleared per call: ``live_events`` gives the mask).
    """
    P: torch.Tensor | None
    R: torch.Tensor | None
    M: torch.Tensor | None
    valid: torch.Tensor | None
    n_events: torch.Tensor | None
    ev_int: torch.Tensor | None
    ev_real: torch.Tensor | None


def live_events(n_events: torch.Tensor, E: int) -> torch.Tensor:
    """[B, E] bool mask of the event slots a call wrote (slot j of stream b iff j < n_events[b])."""
    return torch.arange(E, device=n_events.device)[None, :] < n_events.to(torch.int64)[:, None]


def quantize_adc(samples, full_scale: float, bits: int = ADC_BITS):
    """Simulate ADC quantization with the given full-scale range (sync_aa.py:263-291): per
    component round(clip(v / fs, -1, 1 - 1/L) * L) / L * fs, L = 2^(bits-1), on the GPU, bit for
    bit.  Precision follows numpy's promotion of ``samples.real / full_scale``: complex64 samples
    with a Python-float full_scale stay float32 (complex64 out), otherwise float64 (complex128)."""
    from_numpy = not isinstance(samples, torch.Tensor)
    a = np.asarray(samples) if from_numpy else samples
    if from_numpy:
        rdt = a.real.dtype if np.iscomplexobj(a) else a.dtype
    else:
        rdt = {torch.complex64: np.float32, torch.float32: np.float32}.get(a.dtype, np.float64)
    prec_dt = (np.zeros(1, dtype=rdt) / full_scale).dtype          # numpy 2's promotion, weak scalars
    fp32 = prec_dt == np.float32
    dev = _lib.require_gpu()
    t = torch.as_tensor(a) if from_numpy else a
    t = t.to(device=dev, dtype=torch.complex64 if (fp32 or t.dtype in (torch.complex64, torch.float32))
             else torch.complex128).contiguous()
    out = torch.empty(t.shape, dtype=torch.complex64 if fp32 else torch.complex128, device=dev)
    fmt = _lib.C64 if t.dtype == torch.complex64 else _lib.C128
    _lib.check(_lib.lib().ofs_quantize_adc(fmt, t.data_ptr(), t.numel(), float(full_scale), int(bits),
                                           _lib.FP32 if fp32 else _lib.FP64, out.data_ptr(), _lib.stream_ptr()),
               "ofs_quantize_adc")
    return _lib.to_host(out) if from_numpy else out


PLACEMENTS = ("plain", "contiguous")
AA_PLACEMENTS = PLACEMENTS + ("auto",)


def allocate(dev, specs, placement: str = "plain"):
    """Device buffers for a batch: ``specs`` = list of (shape, dtype) or None.

    placement "plain": one allocation from torch's caching allocator, carved into 2 MiB-aligned
    buffers; "contiguous": every buffer its own physically contiguous block
    (hipExtMallocWithFlags(hipDeviceMallocContiguous)), freed with the tensor.  The headline
    shape (cfg3, 1.6 GB per launch) runs 0.27-0.30 ms with "contiguous" against 0.30-0.33 ms
    "plain" depending on the box; other shapes measured the opposite, hence a
    per-call choice, default "plain".  Raises MemoryError if the driver cannot back a
    contiguous block.
    """
    if placement == "plain":
        return _lib.arena(dev, specs, contiguous=False)
    if placement == "contiguous":
        return [None if sp is None else _lib.arena(dev, [sp], contiguous=True)[0] for sp in specs]
    raise ValueError(f"placement must be one of {PLACEMENTS}, got {placement!r}")


def _run(batch: _lib.Batch, L: int, threshold: float, hysteresis: int, sample_rate: float,
         prec: int, want=("P", "R", "M", "valid"), detect: bool = True, max_events: int = 16,
         placement: str = "plain"):
    dev = batch.data.device
    B, T = batch.B, batch.T
    ct = torch.complex128 if prec == _lib.FP64 else torch.complex64
    rt = torch.float64 if prec == _lib.FP64 else torch.float32
    P, R, M, V = allocate(dev, [((B, T), ct) if "P" in want else None, ((B, T), rt) if "R" in want else None,
                                ((B, T), rt) if "M" in want else None,
                                ((B, T), torch.bool) if "valid" in want else None], placement)
    n_ev = ev_i = ev_r = None
    if detect:
        # counts zeroed (4 B per stream: T = 0 launches nothing); event slots past a stream's count
        # are never written and stay uninitialised (no per-call memset of 2 x B x E x 32 B; readers
        # mask with live_events)
        n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
        ev_i = torch.empty((B, max(max_events, 1), 4), dtype=torch.int64, device=dev)
        ev_r = torch.empty((B, max(max_events, 1), 4), dtype=torch.float64, device=dev)
    rc = _lib.lib().ofs_aa_detect(batch.fmt, batch.data.data_ptr(), B, batch.nb, T, int(L), prec,
                                  _lib.ptr(P), _lib.ptr(R), _lib.ptr(M), _lib.ptr(V), int(detect),
                                  float(threshold), int(hysteresis), float(sample_rate),
                                  int(max_events), _lib.ptr(n_ev), _lib.ptr(ev_i), _lib.ptr(ev_r),
                                  _lib.stream_ptr())
    _lib.check(rc, "ofs_aa_detect")
    return AABatchResult(P, R, M, V, n_ev, ev_i, ev_r)


class AABatchDetector:
    """Preallocated, launch-only form of ``aa_detect_streaming_batched`` (serving / benchmark use).

    Buffers for a fixed shape [B, n_ant, T] are allocated once (``placement``: see
    ``allocate``); ``run()`` enqueues ONE ``ofs_aa_detect`` launch on the current stream and
    returns without a host synchronisation, so back-to-back calls pipeline on the GPU.  Event
    slots are ``max_events`` per stream; ``overflowed()`` (synchronising) reports whether any
    stream produced more (its count stays exact in ``n_events``; the batched function re-runs
    in that case, this class leaves it to the caller).

    ``placement="auto"`` (default) backs the buffers the way measured fastest for the shape: fp32
    (complex64 in) with whole 8 KiB stream rows (T a multiple of 1024) every buffer its own physically
    contiguous block, everything else one plain arena.  Paired A/B, fresh detectors per round
    (tools/place_ab.py, profiles/r04b_placement_ab.jsonl, r04c_placement_ab.jsonl; contiguous / plain):
    cfg3 0.96, two antennas 0.98, T = 4096 0.88, 2 x 4096 0.99 - but the reference's own 2 x 5315
    shape 1.16, 2 x 5316 1.30, 1 x 4095 1.02 (1 x 5315 0.95 is the one row-unaligned shape it helps);
    fp64 contiguous 0.99 vs 0.59 ms (cfg3), cfg2a 0.044 vs 0.030 ms.  When the driver
    cannot back a contiguous block it falls back to "plain".  ``self.placement`` is the placement used.
    """

    def __init__(self, B: int, T: int, n_ant: int = 1, L: int = PREAMBLE_HALF_LEN,
                 threshold: float = DETECT_THRESHOLD, hysteresis: int = DETECT_HYSTERESIS,
                 sample_rate: float = SAMPLE_RATE_HZ, *, precision="fp32", in_dtype=None,
                 outputs=("P", "R", "M"), detect: bool = True, max_events: int = 4,
                 placement: str = "auto", device=None):
        if placement not in AA_PLACEMENTS:
            raise ValueError(f"placement must be one of {AA_PLACEMENTS}, got {placement!r}")
        dev = torch.device(device) if device is not None else _lib.require_gpu()
        _lib.lib()
        prec = _lib.resolve_precision(_lib.Batch(None, _lib.C64, B, n_ant, T, False, False), precision)
        if in_dtype is None:
            in_dtype = torch.complex64 if prec == _lib.FP32 else torch.complex128
        self.fmt = {torch.complex64: _lib.C64, torch.complex128: _lib.C128, torch.int16: _lib.CI16}[in_dtype]
        ct = torch.complex128 if prec == _lib.FP64 else torch.complex64
        rt = torch.float64 if prec == _lib.FP64 else torch.float32
        xshape = (B, n_ant, T, 2) if in_dtype == torch.int16 else (B, n_ant, T)
        want = tuple(outputs)
        if detect and B > 0 and T > 0 and _lib.lib().ofs_aa_plan(self.fmt, prec, n_ant, T, int(L)) == 2:
            want = tuple(set(want) | {"P", "M"})         # tiled general engine: events from P/M in HBM
        specs = [(xshape, in_dtype), ((B, T), ct) if "P" in want else None, ((B, T), rt) if "R" in want else None,
                 ((B, T), rt) if "M" in want else None, ((B, T), torch.bool) if "valid" in want else None]
        used = placement if placement != "auto" else (
            "contiguous" if prec == _lib.FP32 and T % 1024 == 0 else "plain")
        try:
            self.x, P, R, M, V = allocate(dev, specs, used)
        except MemoryError:
            if placement != "auto":
                raise
            used = "plain"                                  # the driver cannot back a contiguous block
            self.x, P, R, M, V = allocate(dev, specs, used)
        placement = used
        E = max(int(max_events), 1)
        n_ev = torch.zeros((B,), dtype=torch.int32, device=dev) if detect else None
        # event slots past a stream's n_events are never written: zero-filled once so a reader
        # never sees uninitialised memory
        ev_i = torch.zeros((B, E, 4), dtype=torch.int64, device=dev) if detect else None
        ev_r = torch.zeros((B, E, 4), dtype=torch.float64, device=dev) if detect else None
        self.result = AABatchResult(P, R, M, V, n_ev, ev_i, ev_r)
        self.B, self.T, self.n_ant, self.L, self.prec, self.max_events = B, T, n_ant, int(L), prec, E
        self.placement, self.device = placement, dev
        self._fn = _lib.lib().ofs_aa_detect
        self._tail = (prec, _lib.ptr(P), _lib.ptr(R), _lib.ptr(M), _lib.ptr(V), int(detect), float(threshold),
                      int(hysteresis), float(sample_rate), E, _lib.ptr(n_ev), _lib.ptr(ev_i), _lib.ptr(ev_r))

    def plan(self) -> int:
        """ofs_aa_plan of this shape (which kernel ``run`` launches)."""
        return int(_lib.lib().ofs_aa_plan(self.fmt, self.prec, self.n_ant, self.T, self.L))

    def run(self, x: torch.Tensor | None = None, stream: int | None = None) -> AABatchResult:
        """Launch on the batch in ``x`` (default: the detector's own input buffer ``self.x``)."""
        x = self.x if x is None else x
        if x.device != self.device or not x.is_contiguous() or x.numel() != self.x.numel() or x.dtype != self.x.dtype:
            raise ValueError("x must be a contiguous device tensor shaped and typed like AABatchDetector.x")
        rc = self._fn(self.fmt, x.data_ptr(), self.B, self.n_ant, self.T, self.L, *self._tail,
                      _lib.stream_ptr() if stream is None else stream)
        _lib.check(rc, "ofs_aa_detect")
        return self.result

    def overflowed(self) -> bool:
        n = self.result.n_events
        return bool(n is not None and n.numel() and int(n.max().item()) > self.max_events)


def aa_detect_streaming_batched(x, L: int = PREAMBLE_HALF_LEN, threshold: float = DETECT_THRESHOLD,
                                hysteresis: int = DETECT_HYSTERESIS,
                                sample_rate: float = SAMPLE_RATE_HZ, *, precision=None,
                                outputs=("P", "R", "M", "valid"), detect: bool = True,
                                max_events: int = 16, placement: str = "plain") -> AABatchResult:
    """Batched [A][A] detector over independent streams x[B, n_ant, T] (or [B, T]).

    Same per-stream semantics as ``aa_detect_streaming``; results stay on the GPU.
    ``precision``: None (fp64 for complex128/int16 input, fp32 for complex64), 'fp32', 'fp64'.
    ``placement``: output backing, "plain" or "contiguous" (see ``allocate``).

    Detect-only calls (``outputs=()``) on the fp32 fast path run their own arithmetic (fp32 row
    scans, 4 samples per lane; the storing call scans in fp64): their events can differ from a
    storing call's, but only where the reference's own float64 decision is a near-tie (a metric
    within 1e-6 of the threshold, or two |P|^2 candidates within 1e-5 relative in a gate) -
    tests/test_gpu_detect_only.py::test_default_detect_only_vs_default_full_near_threshold.
    """
    batch = _lib.as_batch(x, batched=True)
    prec = _lib.resolve_precision(batch, precision)
    want = tuple(outputs)
    # events on a multi-tile stream of the general engine (plan 2) are found in a second pass
    # over P/M in HBM; every other plan keeps them on chip, so detect-only skips those stores
    if detect and batch.T > 0 and _lib.lib().ofs_aa_plan(batch.fmt, prec, batch.nb, batch.T, int(L)) == 2:
        want = tuple(sorted(set(want) | {"P", "M"}, key=["P", "R", "M", "valid"].index))
    res = _run(batch, L, threshold, hysteresis, sample_rate, prec, want, detect, max_events, placement)
    if detect and batch.B > 0 and batch.T > 0:
        worst = int(res.n_events.max().item())
        if worst > max_events:
            res = _run(batch, L, threshold, hysteresis, sample_rate, prec, want, detect, worst, placement)
    for name in ("P", "R", "M", "valid"):
        if name not in outputs:
            setattr(res, name, None)
    return res


def aa_detect_streaming(
    rx_samples: np.ndarray,
    L: int = PREAMBLE_HALF_LEN,
    threshold: float = DETECT_THRESHOLD,
    hysteresis: int = DETECT_HYSTERESIS,
    sample_rate: float = SAMPLE_RATE_HZ,
    *,
    precision=None,
) -> AADetectionResult:
    """Streaming [A][A] detector with multi-antenna support (drop-in for sync_aa.py:421-571).

    rx_samples: (num_antennas, num_samples) or (num_samples,).  Returns AADetectionResult
    with numpy state arrays (torch input -> torch device tensors).
    """
    batch = _lib.as_batch(rx_samples, batched=False)
    prec = _lib.resolve_precision(batch, precision)
    num_antennas = batch.nb
    T = batch.T
    if T == 0:
        empty = AADetectorState(P=np.zeros(0, np.complex128), R=np.zeros(0), M=np.zeros(0),
                                valid=np.zeros(0, bool))
        return AADetectionResult(events=[], state=empty, num_antennas=num_antennas)
    max_ev = 16
    res = _run(batch, L, threshold, hysteresis, sample_rate, prec, detect=True, max_events=max_ev)
    n = int(res.n_events[0].item())
    if n > max_ev:
        res = _run(batch, L, threshold, hysteresis, sample_rate, prec, detect=True, max_events=n)
    ev_i = res.ev_int[0, :n].cpu().numpy()
    ev_r = res.ev_real[0, :n].cpu().numpy()
    events = [
        AADetectionEvent(peak_index=int(a[0]), P_at_peak=complex(r[0], r[1]), M_at_peak=float(r[2]),
                         gate_start=int(a[1]), gate_end=int(a[2]), cfo_hz=float(r[3]),
                         frame_start=int(a[3]))
        for a, r in zip(ev_i, ev_r)
    ]
    if batch.from_numpy:
        state = AADetectorState(P=_lib.to_host(res.P[0], np.complex128), R=_lib.to_host(res.R[0], np.float64),
                                M=_lib.to_host(res.M[0], np.float64), valid=_lib.to_host(res.valid[0]))
    else:
        state = AADetectorState(P=res.P[0], R=res.R[0], M=res.M[0], valid=res.valid[0])
    return AADetectionResult(events=events, state=state, num_antennas=num_antennas)
