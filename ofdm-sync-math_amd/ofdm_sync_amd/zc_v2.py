"""Drop-in for the FPGA-style ZC matched-filter detector of ``zc_v2.py``.

matched_filter_correlation  zc_v2.py:244-254  -> ofs_zc_correlate (OFS_ZC_RAW)
normalize_correlation       zc_v2.py:257-271  -> ofs_zc_correlate (OFS_ZC_NORMALIZE)
zc_streaming_detection      zc_v2.py:300-346  -> ofs_zc_detect (flags only)
detect_zc_peaks             zc_v2.py:374-446  -> ofs_zc_gate
detect_zc_preamble          zc_v2.py:452-519  -> ofs_zc_correlate (OFS_ZC_V2 / OFS_ZC_SUM,
                                                 |corr| fused) + ofs_zc_detect (CFAR + gate fused)
The correlation is an LDS-tiled direct sum in fp64 (csrc/corr.hip) or, from 256 taps, FFT
overlap-save (csrc/zc_fftcorr.hip); the CFAR running sum is the reference's sequential float64
recursion evaluated one lane per stream and the gate a closed-form machine over 64-sample rows
(csrc/zc_cfar.hip; hysteresis < 64 and detect_zc_peaks on a given state: one wave per stream).
``build_pss_symbol`` is host-side setup of the reference waveform (zc_v2.py:170-185).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

N_FFT = 2048                                  # core.py:6
CYCLIC_PREFIX = 512                           # core.py:8
PSS_LENGTH = 62                               # zc_v2.py:115
PSS_ROOT = 25                                 # zc_v2.py:116
CORR_WINDOW_SIZE = N_FFT                      # zc_v2.py:123
THRESH_FRAC_BITS = 15                         # zc_v2.py:126
THRESH_VALUE = int(4.0 * (1 << THRESH_FRAC_BITS) / CORR_WINDOW_SIZE)   # zc_v2.py:143
MIN_CORR_MAG = 0.3                            # zc_v2.py:147
HYSTERESIS = 256                              # zc_v2.py:151

OFS_ZC_RAW, OFS_ZC_V2, OFS_ZC_COMBINED, OFS_ZC_NORMALIZE, OFS_ZC_SUM = 0, 1, 2, 3, 4


def centered_subcarrier_indices(width: int) -> np.ndarray:
    half = width // 2
    return np.concatenate((np.arange(-half, 0), np.arange(1, half + 1)))


def generate_zadoff_chu(root: int, length: int) -> np.ndarray:
    n = np.arange(length)
    return np.exp(-1j * np.pi * root * n * (n + 1) / length)


def build_pss_symbol(include_cp: bool = False, *, n_fft: int | None = None,
                     cyclic_prefix: int | None = None) -> np.ndarray:
    """ZC on the centered bins, unit-power time symbol (zc_v2.py:170-185, core.py:21-47).

    ``n_fft`` / ``cyclic_prefix`` default to this module's N_FFT / CYCLIC_PREFIX read at call
    time (the reference's module globals); passing them never mutates the globals."""
    N = N_FFT if n_fft is None else int(n_fft)
    cp = CYCLIC_PREFIX if cyclic_prefix is None else int(cyclic_prefix)
    idx = centered_subcarrier_indices(PSS_LENGTH)
    spec = np.zeros(N, dtype=complex)
    spec[(N // 2 + idx) % N] = generate_zadoff_chu(PSS_ROOT, PSS_LENGTH)
    sym = np.fft.ifft(np.fft.ifftshift(spec))
    p = np.mean(np.abs(sym) ** 2)
    if p != 0:
        sym = sym / np.sqrt(p)
    if include_cp and cp > 0:
        sym = np.concatenate((sym[-cp:], sym))
    return sym


@dataclass
class ZCDetectionState:
    corr_mag: np.ndarray
    local_sum: np.ndarray
    corr_scaled: np.ndarray
    thresh_scaled: np.ndarray
    above_threshold: np.ndarray
    metric_valid: np.ndarray


@dataclass
class ZCDetectionEvent:
    peak_index: int
    peak_value: float
    gate_start: int
    gate_end: int
    detected_start: int


@dataclass
class ZCDetectionResult:
    events: list[ZCDetectionEvent]
    gate_mask: np.ndarray
    state: ZCDetectionState


def _ref_host(reference) -> np.ndarray:
    """The reference taps as a contiguous complex128 host array (a device tensor is copied: a
    few KB, once per call).  Everything that identifies a reference - the plan-cache key, the
    energy - is computed from these bytes, never from a device address: the caching allocator
    hands a freed reference's address to the next one, so (data_ptr, _version) does not
    identify contents."""
    if isinstance(reference, torch.Tensor):
        return np.ascontiguousarray(reference.detach().to(torch.complex128).cpu().numpy().reshape(-1))
    return np.ascontiguousarray(np.asarray(reference, dtype=np.complex128).reshape(-1))


def _ref_key(r_host: np.ndarray) -> tuple:
    """Content identity of a reference for the plan cache: digest of its complex128 bytes."""
    import hashlib
    return (hashlib.sha1(r_host.tobytes()).hexdigest(), r_host.size)


def _ref_dev(reference, r_host: np.ndarray, dev):
    """(device complex128 taps, energy); energy as the reference computes it (zc_v2.py:263)."""
    energy = float(np.sum(np.abs(r_host) ** 2))
    if isinstance(reference, torch.Tensor):
        return reference.to(device=dev, dtype=torch.complex128).contiguous().reshape(-1), energy
    return torch.from_numpy(r_host).to(dev), energy


class MatchedFilter:
    """A prepared reference for the batched correlation / detection entry points
    (``correlate_batched``, ``detect_zc_preamble_batched``): its complex128 taps (host copy and a
    device copy), its energy (zc_v2.py:263) and its content key for the FFT plan cache are computed
    ONCE here.  A raw device tensor passed as ``reference`` is copied to the host and hashed on
    every call (a stream synchronisation per call); a MatchedFilter skips that.  The taps are a
    snapshot: later writes to the tensor it was built from do not reach it."""

    def __init__(self, reference, device=None):
        self.host = _ref_host(reference)
        self.key = _ref_key(self.host)
        self.energy = float(np.sum(np.abs(self.host) ** 2))
        self.device = torch.device(device) if device is not None else _lib.require_gpu()
        self.taps = torch.from_numpy(self.host).to(self.device)

    def __len__(self) -> int:
        return int(self.host.size)

    def taps_on(self, dev) -> torch.Tensor:
        return self.taps if self.taps.device == torch.device(dev) else self.taps.to(dev)

    def correlate(self, x, mode: int = None, **kw):
        """correlate_batched(x, self, mode, ...): mode defaults to OFS_ZC_V2 (|corr| normalised)."""
        return correlate_batched(x, self, OFS_ZC_V2 if mode is None else mode, **kw)


class MFPlan:
    """FFT overlap-save matched-filter plan (ofs_zc_mf_plan_create) for one reference and one
    batch shape [B, n_branch, T]: the rocFFT plans, the reference spectrum and the plan's rocFFT
    execution info.  The per-call scratch (the blocks' spectra) and rocFFT work buffer are NOT
    part of the plan: ``run`` takes them from torch's stream-ordered caching allocator, so calls
    on different streams never share a buffer.  ``run`` holds the plan's lock while it sets the
    execution info's stream / work buffer and enqueues (the C plan is one caller at a time)."""

    def __init__(self, reference, B: int, nb: int, T: int, dev, M: int = 0):
        import ctypes
        import threading
        r = _ref_host(reference)
        self._lib = _lib.lib()
        h, wb, sb = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_size_t()
        _lib.check(self._lib.ofs_zc_mf_plan_create(r.ctypes.data, r.size, int(B), int(nb), int(T), int(M),
                                                  ctypes.byref(h), ctypes.byref(wb), ctypes.byref(sb)),
                   "ofs_zc_mf_plan_create")
        self.handle = h.value
        self.shape = (int(B), int(nb), int(T))
        self.scratch_bytes, self.work_bytes = max(int(sb.value), 1), int(wb.value)
        self.device = dev
        self._lock = threading.Lock()

    def run(self, batch, energy: float, mode: int, corr, mag) -> None:
        scratch = torch.empty((self.scratch_bytes,), dtype=torch.uint8, device=self.device)
        work = torch.empty((self.work_bytes,), dtype=torch.uint8, device=self.device) if self.work_bytes else None
        with self._lock:
            rc = self._lib.ofs_zc_correlate_fft(self.handle, batch.fmt, batch.data.data_ptr(), batch.B, batch.nb,
                                                batch.T, energy, int(mode), _lib.ptr(corr), _lib.ptr(mag),
                                                scratch.data_ptr(), _lib.ptr(work), _lib.stream_ptr())
        _lib.check(rc, "ofs_zc_correlate_fft")

    def __del__(self):
        h, self.handle = getattr(self, "handle", None), None
        if h:
            self._lib.ofs_zc_mf_plan_destroy(h)


_mf_plans: dict = {}
FFT_MIN_TAPS = 256          # the FFT path from this reference length on (direct sums below)
_NO_PLAN = object()         # cached "this shape has no FFT plan" (OFS_ETOOLONG)


def _mf_plan(reference, key, B, nb, T, dev):
    """The cached plan for (reference, shape, device), or None when the overlap-save extract
    cannot hold this shape's per-block energy prefixes in LDS (OFS_ETOOLONG: many branches or
    long references).  Plans hold no per-call buffers, so the cache pins only rocFFT plans."""
    k = (key, int(B), int(nb), int(T), str(dev))
    p = _mf_plans.get(k)
    if p is None:
        if len(_mf_plans) >= 8:
            _mf_plans.clear()
        try:
            p = MFPlan(reference, B, nb, T, dev)
        except RuntimeError as e:
            if "status -2)" not in str(e):                 # only OFS_ETOOLONG means "no plan"
                raise
            p = _NO_PLAN
        _mf_plans[k] = p
    return None if p is _NO_PLAN else p


def correlate_batched(x, reference, mode: int, corr_in=None, want_corr=True, want_mag=False, method: str = "auto"):
    """Correlation of x[B, n_branch, T] with `reference` -> (corr, corr_mag) device tensors.

    method "direct": ofs_zc_correlate (O(N) MACs per output, fp64); "fft": ofs_zc_correlate_fft
    (overlap-save through rocFFT, fp64; raises if the shape has no plan); "auto": the FFT path
    for references of >= FFT_MIN_TAPS taps (measured 2048 taps: DESIGN.md §4.5b) in every mode
    but OFS_ZC_NORMALIZE, falling back to the direct sums for shapes the overlap-save extract
    cannot hold (ofs_zc_mf_plan_create -> OFS_ETOOLONG: e.g. 4 branches at N = 2048).
    ``reference``: taps (numpy / tensor) or a MatchedFilter (no per-call host copy or hashing)."""
    batch = _lib.as_batch(x, batched=True)
    dev = batch.data.device
    mf = reference if isinstance(reference, MatchedFilter) else None
    r_host = mf.host if mf is not None else _ref_host(reference)
    energy = mf.energy if mf is not None else float(np.sum(np.abs(r_host) ** 2))   # zc_v2.py:263
    N = int(r_host.size)
    nout = batch.T + N - 1
    shape = (batch.B, batch.nb, nout) if mode == OFS_ZC_RAW else (batch.B, nout)
    corr = torch.empty(shape, dtype=torch.complex128, device=dev) if want_corr else None
    mag = torch.empty(shape, dtype=torch.float64, device=dev) if want_mag else None
    if method not in ("auto", "direct", "fft"):
        raise ValueError("method must be 'auto', 'direct' or 'fft'")
    use_fft = mode != OFS_ZC_NORMALIZE and batch.B > 0 and batch.T > 0 and (
        method == "fft" or (method == "auto" and N >= FFT_MIN_TAPS))
    if use_fft:
        plan = _mf_plan(r_host, mf.key if mf is not None else _ref_key(r_host), batch.B, batch.nb, batch.T, dev)
        if plan is not None:
            plan.run(batch, energy, mode, corr, mag)
            return corr, mag
        if method == "fft":
            raise RuntimeError(f"ofs_zc_mf_plan_create: no overlap-save plan for {batch.nb} branches x "
                               f"{N} taps (extract LDS); use method='direct' (status -2)")
    # the direct sums read the taps on the device
    ref = mf.taps_on(dev) if mf is not None else _ref_dev(reference, r_host, dev)[0]
    ci = None
    if mode == OFS_ZC_NORMALIZE:
        ci = torch.as_tensor(corr_in).to(device=dev, dtype=torch.complex128).reshape(batch.B, nout).contiguous()
    rc = _lib.lib().ofs_zc_correlate(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T,
                                     ref.data_ptr(), N, energy, int(mode), _lib.ptr(ci), _lib.ptr(corr),
                                     _lib.ptr(mag), _lib.stream_ptr())
    _lib.check(rc, "ofs_zc_correlate")
    return corr, mag


def matched_filter_correlation(rx_samples, reference):
    """np.convolve(rx, conj(reference[::-1]), 'full') on the GPU (zc_v2.py:244-254)."""
    from_numpy = not isinstance(rx_samples, torch.Tensor)
    x = rx_samples if not from_numpy else np.asarray(rx_samples)
    if x.ndim != 1:
        raise ValueError("matched_filter_correlation takes one branch (1-D samples)")
    corr, _ = correlate_batched(x[None, None], reference, OFS_ZC_RAW)
    return _lib.to_host(corr[0, 0], np.complex128) if from_numpy else corr[0, 0]


def normalize_correlation(corr, rx_samples, reference):
    """corr / (sqrt(E_ref) * sqrt(max(sliding |rx|^2 over len(ref), 1e-12))) (zc_v2.py:257-271)."""
    from_numpy = not isinstance(rx_samples, torch.Tensor)
    x = rx_samples if not from_numpy else np.asarray(rx_samples)
    if x.ndim != 1:
        raise ValueError("normalize_correlation takes one branch (1-D samples)")
    out, _ = correlate_batched(x[None, None], reference, OFS_ZC_NORMALIZE, corr_in=corr)
    return _lib.to_host(out[0], np.complex128) if from_numpy else out[0]


def _detect_run(mag: torch.Tensor, window_size, thresh_value, thresh_frac_bits, min_corr_mag,
                reference_length, hysteresis, max_events, want_state=True):
    B, n = mag.shape
    dev = mag.device
    f64 = lambda: torch.empty((B, n), dtype=torch.float64, device=dev)   # noqa: E731
    u8 = lambda: torch.empty((B, n), dtype=torch.uint8, device=dev)      # noqa: E731
    st = dict(local_sum=f64(), corr_scaled=f64(), thresh_scaled=f64(), above_threshold=u8(),
              metric_valid=u8()) if want_state else {}
    gate = u8()
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    E = max(int(max_events), 1)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_v = torch.empty((B, E), dtype=torch.float64, device=dev)
    g = st.get
    rc = _lib.lib().ofs_zc_detect(mag.data_ptr(), B, n, int(window_size), int(thresh_value),
                                  int(thresh_frac_bits), float(min_corr_mag), int(reference_length),
                                  int(hysteresis), _lib.ptr(g("local_sum")), _lib.ptr(g("corr_scaled")),
                                  _lib.ptr(g("thresh_scaled")), _lib.ptr(g("above_threshold")),
                                  _lib.ptr(g("metric_valid")), gate.data_ptr(), E, n_ev.data_ptr(),
                                  ev_i.data_ptr(), ev_v.data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "ofs_zc_detect")
    return st, gate, n_ev, ev_i, ev_v


def zc_streaming_detection(corr_mag, window_size: int = CORR_WINDOW_SIZE, thresh_value: int = THRESH_VALUE,
                           thresh_frac_bits: int = THRESH_FRAC_BITS,
                           min_corr_mag: float = MIN_CORR_MAG) -> ZCDetectionState:
    """Adaptive-threshold CFAR on |corr| (zc_v2.py:300-346)."""
    from_numpy = not isinstance(corr_mag, torch.Tensor)
    dev = _lib.require_gpu()
    m = torch.as_tensor(np.asarray(corr_mag, np.float64) if from_numpy else corr_mag)
    m = m.to(device=dev, dtype=torch.float64).reshape(1, -1).contiguous()
    st, *_ = _detect_run(m, window_size, thresh_value, thresh_frac_bits, min_corr_mag, 0, 0, 0)
    conv = (lambda t, dt: _lib.to_host(t[0], dt)) if from_numpy else (lambda t, dt: t[0])
    return ZCDetectionState(
        corr_mag=np.asarray(corr_mag, np.float64) if from_numpy else m[0],
        local_sum=conv(st["local_sum"], np.float64), corr_scaled=conv(st["corr_scaled"], np.float64),
        thresh_scaled=conv(st["thresh_scaled"], np.float64),
        above_threshold=conv(st["above_threshold"].bool(), bool),
        metric_valid=conv(st["metric_valid"].bool(), bool))


def _events(n_ev, ev_i, ev_v):
    k = int(n_ev)
    ei = ev_i[:k].cpu().numpy()
    ev = ev_v[:k].cpu().numpy()
    return [ZCDetectionEvent(peak_index=int(r[0]), peak_value=float(v), gate_start=int(r[1]),
                             gate_end=int(r[2]), detected_start=int(r[3])) for r, v in zip(ei, ev)]


def detect_zc_peaks(state: ZCDetectionState, reference_length: int,
                    hysteresis: int = HYSTERESIS) -> ZCDetectionResult:
    """Gate logic and peak tracking on an existing state (zc_v2.py:374-446)."""
    dev = _lib.require_gpu()
    from_numpy = not isinstance(state.corr_mag, torch.Tensor)
    t = lambda a, dt: torch.as_tensor(np.asarray(a) if from_numpy else a).to(device=dev, dtype=dt).reshape(1, -1).contiguous()  # noqa: E731,E501
    mag = t(state.corr_mag, torch.float64)
    ab = t(state.above_threshold, torch.uint8)
    vd = t(state.metric_valid, torch.uint8)
    n = mag.shape[1]
    E = 16
    while True:
        gate = torch.empty((1, n), dtype=torch.uint8, device=dev)
        n_ev = torch.zeros(1, dtype=torch.int32, device=dev)
        ev_i = torch.empty((1, E, 4), dtype=torch.int64, device=dev)
        ev_v = torch.empty((1, E), dtype=torch.float64, device=dev)
        rc = _lib.lib().ofs_zc_gate(mag.data_ptr(), ab.data_ptr(), vd.data_ptr(), 1, n, int(reference_length),
                                    int(hysteresis), gate.data_ptr(), E, n_ev.data_ptr(), ev_i.data_ptr(),
                                    ev_v.data_ptr(), _lib.stream_ptr())
        _lib.check(rc, "ofs_zc_gate")
        k = int(n_ev[0])
        if k <= E:
            break
        E = k
    mask = gate[0].bool()
    return ZCDetectionResult(events=_events(k, ev_i[0], ev_v[0]),
                             gate_mask=_lib.to_host(mask, bool) if from_numpy else mask, state=state)


@dataclass
class ZCBatchResult:
    """Device-resident batched detection: corr_mag and flags [B, T+N-1];
    n_events [B]; events [B, E, 4] = peak_index, gate_start, gate_end, detected_start;
    peak_values [B, E]."""
    corr_mag: torch.Tensor
    state: dict
    gate_mask: torch.Tensor
    n_events: torch.Tensor
    events: torch.Tensor
    peak_values: torch.Tensor


def detect_zc_preamble_batched(x, reference=None, window_size: int = CORR_WINDOW_SIZE,
                               thresh_value: int = THRESH_VALUE, thresh_frac_bits: int = THRESH_FRAC_BITS,
                               min_corr_mag: float = MIN_CORR_MAG, hysteresis: int = HYSTERESIS,
                               normalize: bool = True, max_events: int = 8,
                               want_state: bool = True) -> ZCBatchResult:
    """detect_zc_preamble over x[B, n_branch, T]; everything stays on the device.  ``reference``:
    taps or a MatchedFilter (default: the PSS symbol of build_pss_symbol)."""
    if reference is None:
        reference = build_pss_symbol(include_cp=False)
    ref_len = int(len(reference))
    _, mag = correlate_batched(x, reference, OFS_ZC_V2 if normalize else OFS_ZC_SUM,
                               want_corr=False, want_mag=True)
    E = int(max_events)
    while True:
        st, gate, n_ev, ev_i, ev_v = _detect_run(mag, window_size, thresh_value, thresh_frac_bits,
                                                 min_corr_mag, ref_len, hysteresis, E, want_state)
        worst = int(n_ev.max()) if n_ev.numel() else 0
        if worst <= E:
            break
        E = worst
    return ZCBatchResult(corr_mag=mag, state=st, gate_mask=gate, n_events=n_ev, events=ev_i,
                         peak_values=ev_v)


def detect_zc_preamble(rx_samples, window_size: int = CORR_WINDOW_SIZE, thresh_value: int = THRESH_VALUE,
                       thresh_frac_bits: int = THRESH_FRAC_BITS, min_corr_mag: float = MIN_CORR_MAG,
                       hysteresis: int = HYSTERESIS, normalize: bool = True) -> ZCDetectionResult:
    """Full ZC preamble detection pipeline (zc_v2.py:452-519)."""
    from_numpy = not isinstance(rx_samples, torch.Tensor)
    x = np.asarray(rx_samples) if from_numpy else rx_samples
    if x.ndim == 1:
        x = x[None]
    r = detect_zc_preamble_batched(x[None], None, window_size, thresh_value, thresh_frac_bits,
                                   min_corr_mag, hysteresis, normalize)
    conv = (lambda t, dt: _lib.to_host(t[0], dt)) if from_numpy else (lambda t, dt: t[0])
    st = ZCDetectionState(
        corr_mag=conv(r.corr_mag, np.float64), local_sum=conv(r.state["local_sum"], np.float64),
        corr_scaled=conv(r.state["corr_scaled"], np.float64),
        thresh_scaled=conv(r.state["thresh_scaled"], np.float64),
        above_threshold=conv(r.state["above_threshold"].bool(), bool),
        metric_valid=conv(r.state["metric_valid"].bool(), bool))
    return ZCDetectionResult(events=_events(r.n_events[0], r.events[0], r.peak_values[0]),
                             gate_mask=conv(r.gate_mask.bool(), bool), state=st)
