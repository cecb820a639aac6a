"""Drop-in for the LTE-style frequency-domain ZC metric of ``zc_freq.py``.

compute_frequency_metric (reference: zc_freq.py:62-99) runs on ``ofs_zc_freq_metric``
(csrc/zc_slide.hip, csrc/corr.hip): the 62 template bins of every window's N-point DFT are
produced by a sliding DFT in fp64 (not one FFT per offset); complex64 input returns float32
(window FFTs in fp32 for a few offsets per stream, else the fp64 sliding DFT rounded to fp32).  ``N_FFT`` and
``CYCLIC_PREFIX`` are read from this module's globals at call time, like the reference.
The template helpers are host-side setup of 62 constants (zc_freq.py:37-59).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

N_FFT = 2048            # core.py:6
CYCLIC_PREFIX = 512     # core.py:8
PSS_LENGTH = 62         # zc_freq.py:30
PSS_ROOT = 25           # zc_freq.py:31


def centered_subcarrier_indices(width: int) -> np.ndarray:
    """core.py:13-18: +-1 .. +-width/2, skipping DC."""
    half = width // 2
    return np.concatenate((np.arange(-half, 0), np.arange(1, half + 1)))


def generate_zadoff_chu(root: int, length: int) -> np.ndarray:
    n = np.arange(length)
    return np.exp(-1j * np.pi * root * n * (n + 1) / length)


def make_pss_frequency_template() -> tuple[np.ndarray, np.ndarray, float]:
    """Return (centered_bin_indices, template_bins, template_energy) (zc_freq.py:54-59)."""
    bin_indices = centered_subcarrier_indices(PSS_LENGTH)
    template_bins = generate_zadoff_chu(PSS_ROOT, PSS_LENGTH)
    energy = float(np.sum(np.abs(template_bins) ** 2))
    return bin_indices, template_bins, energy


MAX_GROUP_BRANCHES = 4      # ofs_zc_freq_partial: branches per kernel pass
MAX_GROUP_BINS = 64         # template bins per kernel pass (one lane per bin)


def _run(batch: _lib.Batch, N: int, cp: int, bin_indices, template_bins, template_energy,
         precision=None):
    idx = np.ascontiguousarray(np.asarray(bin_indices).reshape(-1).astype(np.int32))
    tb = np.ascontiguousarray(np.asarray(template_bins, dtype=np.complex128).reshape(-1))
    if np.asarray(bin_indices).ndim != 1 or tb.shape != idx.shape:
        raise ValueError("bin_indices and template_bins must be 1-D of equal length")
    noff = batch.T - (N + cp) + 1
    if noff <= 0:
        raise ValueError("Received stream is shorter than a single OFDM symbol.")
    L = _lib.lib()
    prec = _lib.resolve_precision(batch, precision)     # complex64 -> fp32 result, whatever the offsets
    dev = batch.data.device
    out = torch.empty((batch.B, noff), dtype=torch.float64 if prec == _lib.FP64 else torch.float32, device=dev)
    if idx.size == 0:                                   # no bins: corr 0, energy 0 -> 0 / max(0, eps)
        return out.zero_()
    if batch.nb <= MAX_GROUP_BRANCHES and idx.size <= MAX_GROUP_BINS:
        rc = L.ofs_zc_freq_metric(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T, int(N),
                                  int(cp), prec, int(idx.size), idx.ctypes.data, tb.ctypes.data,
                                  float(template_energy), out.data_ptr(), _lib.stream_ptr())
        _lib.check(rc, "ofs_zc_freq_metric")
        return out
    # any branch count / template length (zc_freq.py:85-97 loops over both): partial sums of the
    # numerator C and the energy D over groups of <= 4 branches x <= 64 bins, one normalisation
    part = torch.empty((batch.B, noff, 3), dtype=torch.float64, device=dev)
    first = True
    for br0 in range(0, batch.nb, MAX_GROUP_BRANCHES):
        ng = min(MAX_GROUP_BRANCHES, batch.nb - br0)
        for j0 in range(0, idx.size, MAX_GROUP_BINS):
            ig = np.ascontiguousarray(idx[j0:j0 + MAX_GROUP_BINS])
            tg = np.ascontiguousarray(tb[j0:j0 + MAX_GROUP_BINS])
            rc = L.ofs_zc_freq_partial(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T, br0, ng,
                                       int(N), int(cp), int(ig.size), ig.ctypes.data, tg.ctypes.data,
                                       0 if first else 1, part.data_ptr(), _lib.stream_ptr())
            _lib.check(rc, "ofs_zc_freq_partial")
            first = False
    _lib.check(L.ofs_zc_freq_finish(part.data_ptr(), batch.B, noff, float(template_energy), prec, out.data_ptr(),
                                    _lib.stream_ptr()), "ofs_zc_freq_finish")
    return out


def compute_frequency_metric(rx_samples, bin_indices, template_bins, template_energy: float, *,
                             precision=None):
    """Evaluate the LTE-style frequency-domain metric across all offsets (zc_freq.py:62-99)."""
    batch = _lib.as_batch(rx_samples, batched=False)
    out = _run(batch, int(N_FFT), int(CYCLIC_PREFIX), bin_indices, template_bins, template_energy,
               precision)
    return _lib.to_host(out[0], np.float64) if batch.from_numpy else out[0]


def compute_frequency_metric_batched(x, bin_indices=None, template_bins=None, template_energy=None,
                                     N: int | None = None, cp: int | None = None, *, precision=None):
    """Batched metric over x[B, n_branch, T] -> device tensor [B, T-(N+cp)+1]: f64 for complex128
    / int16 input (sliding DFT), f32 for complex64 input (window FFT for <= 64 offsets per stream,
    else the fp64 sliding DFT with the metric rounded to f32); ``precision`` overrides."""
    if bin_indices is None:
        bin_indices, template_bins, template_energy = make_pss_frequency_template()
    batch = _lib.as_batch(x, batched=True)
    return _run(batch, int(N_FFT if N is None else N), int(CYCLIC_PREFIX if cp is None else cp),
                bin_indices, template_bins, template_energy, precision)


# ------------------------------------------------------------------------------------------
# rocFFT leg (include/ofdmsync.h ofs_zc_freq_metric_fft): batched rocFFT per offset + HIP
# gather / conj-mul / |.|^2 / normalise kernel + first-argmax kernel.  Writes and re-reads the
# full spectrum, so it is the comparison path for the fused window-FFT kernel above.
# ------------------------------------------------------------------------------------------
class FFTPlan:
    """Caller-owned rocFFT plan for ``n_windows`` windows of ``N`` samples at distance ``T``.
    ``prune_bins`` > 0: pruned output (rocFFT store callback keeps only the template bins; the
    spectrum buffer is then [chunk][prune_bins]).  ``chunk`` windows per rocFFT execution (0: all
    of them); ``self.chunk`` is the spectrum buffer's row count."""

    def __init__(self, precision: int, N: int, n_windows: int, T: int, prune_bins: int = 0, chunk: int = 0,
                 rows_cp: int | None = None):
        """rows_cp not None: a ROWS plan (ofs_zc_fft_plan_create_rows) over n_windows = B * n_branch rows
        of T samples, cp = rows_cp, ``chunk`` rows per execution; every offset of a row group is one
        execution (windows one sample apart), pruned to ``prune_bins`` bins."""
        import ctypes
        self._lib = _lib.lib()
        h = ctypes.c_void_p()
        wb = ctypes.c_size_t()
        if rows_cp is None:
            _lib.check(self._lib.ofs_zc_fft_plan_create3(int(precision), int(N), int(n_windows), int(T),
                                                        int(prune_bins), int(chunk), ctypes.byref(h), ctypes.byref(wb)),
                       "ofs_zc_fft_plan_create3")
        else:
            _lib.check(self._lib.ofs_zc_fft_plan_create_rows(int(precision), int(N), int(rows_cp), int(T), int(n_windows),
                                                            int(chunk), int(prune_bins), ctypes.byref(h),
                                                            ctypes.byref(wb)), "ofs_zc_fft_plan_create_rows")
        self.handle, self.work_bytes = h.value, int(wb.value)
        self.prune_bins = int(prune_bins)
        self.chunk = int(self._lib.ofs_zc_fft_plan_chunk(self.handle))
        self.key = (int(precision), int(N), int(n_windows), int(T), int(prune_bins), int(chunk), rows_cp)

    def __del__(self):
        h, self.handle = getattr(self, "handle", None), None
        if h:
            self._lib.ofs_zc_fft_plan_destroy(h)


_plans: dict = {}


def _plan(precision: int, N: int, n_windows: int, T: int, prune_bins: int = 0, chunk: int = 0,
          rows_cp: int | None = None) -> FFTPlan:
    key = (precision, N, n_windows, T, prune_bins, chunk, rows_cp)
    p = _plans.get(key)
    if p is None:
        if len(_plans) >= 8:
            _plans.clear()
        p = _plans[key] = FFTPlan(precision, N, n_windows, T, prune_bins, chunk, rows_cp)
    return p


ROWS_SPECTRUM_BYTES = 256 << 20     # compact spectrum of one rows-plan execution (rows_per_exec sizing)
ROWS_MIN_OFFSETS = 8                # layout "auto": the rows plan from this many offsets per stream on ...
ROWS_MAX_RATIO = 4                  # ... and only while T <= ROWS_MAX_RATIO x offsets: a rows plan transforms
                                    # about T windows per row where the offsets plan transforms n_off, so
                                    # T / n_off is its extra FFT work (r05c, T 4242 / 1683 offsets = 2.5x:
                                    # rows 20.1 vs offsets 49.2 ms - the launches it saves paid for it)


def rows_per_exec(n_rows: int, n_br: int, T: int, n_bins: int, esz: int) -> int:
    """Rows per rows-plan execution: a spectrum (n_bins per window: the template's when pruned, N when
    dense) of about ROWS_SPECTRUM_BYTES, whole streams."""
    per = max(n_br, (ROWS_SPECTRUM_BYTES // max(1, T * n_bins * esz)) // n_br * n_br)
    return min(per, n_rows)                  # (the gather strides its streams over gridDim.y: no 65535 cap)


def pick_rows_layout(layout: str, prunable: bool, chunk, T: int, n_off: int, rows_per_execution=None) -> bool:
    """True when compute_frequency_metric_rocfft_batched takes the rows plan: layout "rows"; or "auto"
    with ``rows_per_execution`` given (it sizes only the rows plan); or "auto" with a prunable template,
    no ``chunk`` (it counts windows of the offsets layout), at least ROWS_MIN_OFFSETS offsets and
    T <= ROWS_MAX_RATIO x n_off.  Each size argument is refused where its layout is not the one taken."""
    if layout not in ("auto", "offsets", "rows"):
        raise ValueError("layout must be 'auto', 'offsets' or 'rows'")
    if chunk and rows_per_execution:
        raise ValueError("chunk (offsets layout) and rows_per_execution (rows layout) exclude each other")
    if layout == "offsets" and rows_per_execution:
        raise ValueError("layout='offsets' takes chunk; rows_per_execution sizes the rows layout")
    rows = layout == "rows" or (layout == "auto" and (bool(rows_per_execution) or (
        prunable and chunk is None and n_off >= ROWS_MIN_OFFSETS and T <= ROWS_MAX_RATIO * n_off)))
    if rows and not prunable:
        raise ValueError("the rows layout needs a prunable template (N a power of two <= 4096, distinct bins)")
    if rows and chunk:
        raise ValueError("layout='rows' takes rows_per_execution; chunk counts windows of the offsets layout")
    return rows


def default_chunk(n_windows: int, n_br: int, N: int, esz: int) -> int:
    """Windows per rocFFT execution for the dense leg: a spectrum buffer of about CHUNK_BYTES
    (a multiple of n_br), so it stays in the 256 MiB Infinity Cache between the FFT and the gather."""
    per = max(n_br, (CHUNK_BYTES // (N * esz)) // n_br * n_br)
    return 0 if per >= n_windows else per


CHUNK_BYTES = 64 << 20


def compute_frequency_metric_rocfft_batched(x, bin_indices=None, template_bins=None, template_energy=None,
                                            N: int | None = None, cp: int | None = None, *,
                                            return_peak: bool = False, pruned: bool = False,
                                            chunk: int | None = None, layout: str = "auto",
                                            rows_per_execution: int | None = None):
    """compute_frequency_metric (zc_freq.py:62-99) over x[B, n_branch, T] through rocFFT: one
    batched FFT of every stream/branch window per offset, then the 62-bin gather and metric.
    complex64 input -> f32 metric, complex128 -> f64.  With ``return_peak`` also returns the
    per-stream ``peak_index`` (int64, np.argmax of zc_freq.py:144) and peak value (f64).
    ``pruned`` (N a power of two <= 4096, distinct bins): rocFFT's store callback keeps only the
    template bins, so no dense spectrum is written (1.03x the algorithmic bytes instead of 2.02x);
    measured 2.3x SLOWER on cfg5 (34.2 vs 15.0 ms: rocFFT's callback kernel calls the store
    through a function pointer per element, and each execution blocks the host on a synchronous
    hipMemcpyFromSymbol), hence off by default in both layouts.
    ``chunk``: windows per rocFFT execution (None or 0: one execution over the whole batch;
    ``default_chunk`` sizes one for the Infinity Cache); the spectrum scratch is [chunk][N].  Chunking
    keeps the spectrum round trip on-die but measured neutral on cfg5 (17.5 vs 17.7 ms): rocFFT's
    own 4096-point kernel, not HBM, bounds the leg.
    ``layout``: "offsets" - one rocFFT execution (+ gather) per offset, as above; "rows" - one execution
    per group of rows covering every offset of them (windows one sample apart, ofs_zc_fft_plan_create_rows;
    dense spectrum rows, or compact ones through the callback with ``pruned``), 2 launches per row group
    instead of 2 per offset - the form for the
    reference's own sliding shape (thousands of offsets per stream); "auto": "rows" when the template is
    prunable, ``chunk`` is not given, there are at least ROWS_MIN_OFFSETS offsets per stream and
    T <= ROWS_MAX_RATIO x offsets (the rows plan's extra FFT work, T / offsets, stays small), else
    "offsets".  ``rows_per_execution``: rows (stream x branch) per rows-plan execution (None or 0:
    ``rows_per_exec`` sizes a ~256 MiB spectrum; given under "auto", it selects the rows layout); ``chunk``
    is the offsets layout's windows per execution: each is refused with the other layout."""
    if bin_indices is None:
        bin_indices, template_bins, template_energy = make_pss_frequency_template()
    batch = _lib.as_batch(x, batched=True)
    if batch.fmt == _lib.CI16:
        raise ValueError("the rocFFT leg takes complex64 or complex128 input")
    N = int(N_FFT if N is None else N)
    cp = int(CYCLIC_PREFIX if cp is None else cp)
    idx = np.ascontiguousarray(np.asarray(bin_indices).astype(np.int32))
    tb = np.ascontiguousarray(np.asarray(template_bins, dtype=np.complex128))
    if idx.ndim != 1 or tb.shape != idx.shape or not 0 < idx.size <= 64:
        raise ValueError("bin_indices and template_bins must be 1-D of equal length (1..64)")
    noff = batch.T - (N + cp) + 1
    if noff <= 0:
        raise ValueError("Received stream is shorter than a single OFDM symbol.")
    prec = _lib.FP32 if batch.fmt == _lib.C64 else _lib.FP64
    dev = batch.data.device
    if batch.B == 0:                                   # empty batch: nothing to transform
        out = torch.empty((0, noff), dtype=torch.float32 if prec == _lib.FP32 else torch.float64, device=dev)
        if return_peak:
            return (out, torch.empty((0,), dtype=torch.int64, device=dev),
                    torch.empty((0,), dtype=torch.float64, device=dev))
        return out
    prunable = N <= 4096 and (N & (N - 1)) == 0 and len(set(idx.tolist())) == idx.size
    rows = pick_rows_layout(layout, prunable, chunk, batch.T, noff, rows_per_execution)
    pruned = bool(pruned) and prunable
    nw = batch.B * batch.nb
    out = torch.empty((batch.B, noff), dtype=torch.float32 if prec == _lib.FP32 else torch.float64, device=dev)
    pk = torch.empty((batch.B,), dtype=torch.int64, device=dev) if return_peak else None
    pv = torch.empty((batch.B,), dtype=torch.float64, device=dev) if return_peak else None
    if rows:
        esz = 8 if prec == _lib.FP32 else 16
        nbin = int(idx.size) if pruned else N               # compact (callback) or dense spectrum rows
        rpe = int(rows_per_execution) if rows_per_execution else rows_per_exec(nw, batch.nb, batch.T, nbin, esz)
        if rpe % batch.nb:
            raise ValueError("rows_per_execution must be a multiple of the branch count")
        plan = _plan(prec, N, nw, batch.T, int(idx.size) if pruned else 0, rpe, rows_cp=cp)
        spec = torch.empty((plan.chunk, nbin), dtype=batch.data.dtype, device=dev)
        work = torch.empty((max(plan.work_bytes, 1),), dtype=torch.uint8, device=dev) if plan.work_bytes else None
        rc = _lib.lib().ofs_zc_freq_metric_fft(plan.handle, batch.fmt, batch.data.data_ptr(), batch.B, batch.nb,
                                               batch.T, N, cp, int(idx.size), idx.ctypes.data, tb.ctypes.data,
                                               float(template_energy), spec.data_ptr(), _lib.ptr(work),
                                               out.data_ptr(), _lib.ptr(pk), _lib.ptr(pv), _lib.stream_ptr())
        _lib.check(rc, "ofs_zc_freq_metric_fft")
        return (out, pk, pv) if return_peak else out
    if chunk is None:
        chunk = 0                                       # one execution (chunking measured neutral)
    if chunk and chunk % batch.nb:
        raise ValueError("chunk must be a multiple of the branch count")
    plan = _plan(prec, N, nw, batch.T, int(idx.size) if pruned else 0, int(chunk))
    spec = torch.empty((plan.chunk, int(idx.size) if pruned else N), dtype=batch.data.dtype, device=dev)
    work = torch.empty((max(plan.work_bytes, 1),), dtype=torch.uint8, device=dev) if plan.work_bytes else None
    rc = _lib.lib().ofs_zc_freq_metric_fft(plan.handle, batch.fmt, batch.data.data_ptr(), batch.B, batch.nb,
                                           batch.T, N, cp, int(idx.size), idx.ctypes.data, tb.ctypes.data,
                                           float(template_energy), spec.data_ptr(), _lib.ptr(work),
                                           out.data_ptr(), _lib.ptr(pk), _lib.ptr(pv), _lib.stream_ptr())
    _lib.check(rc, "ofs_zc_freq_metric_fft")
    return (out, pk, pv) if return_peak else out


def peak_index_batched(metric: torch.Tensor):
    """Per-row first argmax of a device metric [B, n] (zc_freq.py:144 ``int(np.argmax(metric))``),
    on the GPU: returns (index int64 [B], value f64 [B])."""
    if metric.dim() == 1:
        metric = metric[None]
    if metric.dtype not in (torch.float32, torch.float64) or metric.device.type != "cuda":
        raise ValueError("metric must be a float32/float64 CUDA tensor")
    metric = metric.contiguous()
    B, n = metric.shape
    idx = torch.empty((B,), dtype=torch.int64, device=metric.device)
    val = torch.empty((B,), dtype=torch.float64, device=metric.device)
    if n == 0:
        raise ValueError("attempt to get argmax of an empty sequence")
    prec = _lib.FP32 if metric.dtype == torch.float32 else _lib.FP64
    _lib.check(_lib.lib().ofs_row_argmax(prec, metric.data_ptr(), B, n, idx.data_ptr(), val.data_ptr(),
                                         _lib.stream_ptr()), "ofs_row_argmax")
    return idx, val
