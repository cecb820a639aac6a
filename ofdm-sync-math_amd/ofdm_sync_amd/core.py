"""Drop-in for the CP-correlation CFO estimators of ``core.py`` (reference: core.py:179-336):
estimate_cfo_from_cp, estimate_cfo_from_cp_robust, estimate_cfo_from_cp_peak[_with_index],
find_cp_start_via_corr; plus the receiver back-end chain that sc.run_simulation runs after sync
(sc.py:274-311: CFO removal, pilot FFT, LS channel estimate, phase-slope timing, equalisation,
gain alignment, EVM) as one batched kernel (receiver_backend[_batched]).

The builders and plotting of the reference's core.py are out of scope.
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


# ---------------------------------------------------------------------------------------------
# receiver back-end after sync (the inline chain of sc.run_simulation, sc.py:274-311) ->
# ofs_rx_backend
# ---------------------------------------------------------------------------------------------
def centered_subcarrier_indices(width: int) -> np.ndarray:
    """Subcarrier indices symmetric around DC, skipping 0 (core.py:13-18)."""
    half = width // 2
    return np.concatenate((np.arange(-half, 0), np.arange(1, half + 1)))


def receiver_backend_batched(x, pilot_start, data_start, pilot_used, data_used, *, n_fft: int = N_FFT,
                             cp_len: int = CYCLIC_PREFIX, fs_hz: float = SAMPLE_RATE_HZ, bins=None,
                             cfo_hz=None) -> dict:
    """Per frame of x[B, n_branch, T]: CP CFO estimate at the pilot (unless cfo_hz [B] is given),
    CFO removal + branch mean, pilot FFT -> LS channel estimate -> phase-slope timing, data
    FFT -> equalise -> complex-gain alignment -> EVM.  pilot_used / data_used: [n_used] (shared)
    or [B, n_used] known symbols.  Returns device tensors: cfo [B], h [B, n_used], xa [B, n_used],
    gain [B] complex, evm, evm_db, slope, sto [B]."""
    batch = _lib.as_batch(x, batched=True)
    dev = batch.data.device
    k = centered_subcarrier_indices(NUM_ACTIVE_SUBCARRIERS) if bins is None else np.asarray(bins)
    U = int(k.size)

    def dev_i64(v):
        t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
        t = t.to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        if t.numel() == 1 and batch.B > 1:
            t = t.expand(batch.B).contiguous()
        if t.numel() != batch.B:
            raise ValueError("one start per frame expected")
        return t

    def dev_ref(v):
        t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v, dtype=np.complex128))
        t = t.to(device=dev, dtype=torch.complex128).contiguous()
        if t.shape[-1] != U or t.dim() > 2 or (t.dim() == 2 and t.shape[0] != batch.B):
            raise ValueError("known symbols must be [n_used] or [B, n_used]")
        return t, (U if t.dim() == 2 else 0)

    ps, ds = dev_i64(pilot_start), dev_i64(data_start)
    pil, pst = dev_ref(pilot_used)
    dat, dst = dev_ref(data_used)
    kb = torch.as_tensor(k.astype(np.int32)).to(dev)
    cin = None if cfo_hz is None else torch.as_tensor(np.asarray(cfo_hz, np.float64)).to(dev).reshape(-1).contiguous()
    B = batch.B
    f64 = lambda: torch.empty((B,), dtype=torch.float64, device=dev)   # noqa: E731
    out = dict(cfo=f64(), h=torch.empty((B, U), dtype=torch.complex128, device=dev),
               xa=torch.empty((B, U), dtype=torch.complex128, device=dev),
               gain=torch.empty((B,), dtype=torch.complex128, device=dev), evm=f64(), evm_db=f64(), slope=f64(),
               sto=f64())
    rc = _lib.lib().ofs_rx_backend(batch.fmt, batch.data.data_ptr(), B, batch.nb, batch.T, int(n_fft), int(cp_len),
                                   float(fs_hz), ps.data_ptr(), ds.data_ptr(), _lib.ptr(cin), U, kb.data_ptr(),
                                   pil.data_ptr(), pst, dat.data_ptr(), dst, out["cfo"].data_ptr(),
                                   out["h"].data_ptr(), out["xa"].data_ptr(), out["gain"].data_ptr(),
                                   out["evm"].data_ptr(), out["evm_db"].data_ptr(), out["slope"].data_ptr(),
                                   out["sto"].data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "ofs_rx_backend")
    return out


def receiver_backend(rx, pilot_cp_start: int, data_cp_start: int, pilot_used, data_used, *, cfo_hz=None,
                     n_fft: int = N_FFT, cp_len: int = CYCLIC_PREFIX, fs_hz: float = SAMPLE_RATE_HZ) -> dict:
    """One frame (1-D or [branches, T]) through the back-end chain of sc.run_simulation
    (sc.py:274-311); numpy / Python scalars out, keys as receiver_backend_batched."""
    a = rx if isinstance(rx, torch.Tensor) else np.asarray(rx)
    x = a[None] if a.ndim == 1 else a
    out = receiver_backend_batched(x[None], [pilot_cp_start], [data_cp_start], pilot_used, data_used,
                                   n_fft=n_fft, cp_len=cp_len, fs_hz=fs_hz,
                                   cfo_hz=None if cfo_hz is None else [cfo_hz])
    res = {}
    for key, v in out.items():
        v = v[0].cpu()
        res[key] = v.numpy() if v.dim() else (complex(v.item()) if v.is_complex() else float(v.item()))
    return res


# ---------------------------------------------------------------------------------------------
# The back-end helpers one by one (core.py:123-138, 171-176, 339-370, 443-469), as the reference
# drivers call them (sc.py:274-311).  Each has the reference's name, signature and return
# convention (numpy in -> numpy out; torch in -> device tensors) and runs on the GPU; the
# *_batched forms take [B, n] device rows.  The fused chain above stays the fast path.
# Precision: every helper computes in fp64 and returns complex128 / float64 whatever the input
# precision (the reference's drivers hand these helpers complex128 arrays; for complex64 input
# numpy would compute and return complex64 - the fp64 result is the more accurate of the two).
# ---------------------------------------------------------------------------------------------
def _rows(a, dev, dtype=torch.complex128):
    """(device tensor [B, n] of `dtype`, was_numpy, original ndim) for 1-D or 2-D input."""
    from_numpy = not isinstance(a, torch.Tensor)
    t = torch.as_tensor(np.asarray(a)) if from_numpy else a
    nd = t.dim()
    if nd not in (1, 2):
        raise ValueError("expected a 1-D vector or [B, n] rows")
    t = t.to(device=dev, dtype=dtype)
    return (t[None] if nd == 1 else t).contiguous(), from_numpy, nd


def _ref_rows(ref, B, n, dev):
    """A reference operand broadcast like numpy against [B, n] rows: [n] shared (stride 0) or [B, n]."""
    r = torch.as_tensor(np.asarray(ref)) if not isinstance(ref, torch.Tensor) else ref
    r = r.to(device=dev, dtype=torch.complex128).contiguous()
    if r.dim() == 1 and r.shape[0] == n:
        return r, 0
    if r.dim() == 2 and tuple(r.shape) == (B, n):
        return r, n
    raise ValueError(f"operands could not be broadcast together with shapes {(B, n)} {tuple(r.shape)}")


def _out(t, from_numpy, nd):
    t = t if nd == 2 else t[0]
    return _lib.to_host(t) if from_numpy else t


def apply_cfo_batched(x, cfo_hz, fs_hz: float) -> torch.Tensor:
    """core.apply_cfo per stream of x[B, n_branch, T] with cfo_hz [B] (or a scalar) -> complex128."""
    batch = _lib.as_batch(x, batched=True)
    dev = batch.data.device
    c = torch.as_tensor(np.asarray(cfo_hz, np.float64) if not isinstance(cfo_hz, torch.Tensor) else cfo_hz)
    c = c.to(device=dev, dtype=torch.float64).reshape(-1)
    if c.numel() == 1 and batch.B != 1:
        c = c.expand(batch.B)
    c = c.contiguous()
    if c.numel() != batch.B:
        raise ValueError("one cfo per stream expected")
    out = torch.empty((batch.B, batch.nb, batch.T), dtype=torch.complex128, device=dev)
    _lib.check(_lib.lib().ofs_apply_cfo(batch.fmt, batch.data.data_ptr(), batch.B, batch.nb, batch.T, c.data_ptr(),
                                        float(fs_hz), out.data_ptr(), _lib.stream_ptr()), "ofs_apply_cfo")
    return out


def apply_cfo(samples, cfo_hz: float, fs_hz: float):
    """Apply a carrier frequency offset to 1D or 2D samples (core.py:123-138): axis 0 of a 2-D
    input is branches, all rotated by the same tone exp(i 2 pi cfo n / fs)."""
    from_numpy = not isinstance(samples, torch.Tensor)
    a = np.asarray(samples) if from_numpy else samples
    if a.ndim not in (1, 2):
        raise ValueError("samples must be 1D or 2D")
    if from_numpy and not np.iscomplexobj(a):
        a = a.astype(np.complex128)
    elif not from_numpy and not a.is_complex():
        a = a.to(torch.complex128)
    x = a[None] if a.ndim == 1 else a
    out = apply_cfo_batched(x[None], [float(cfo_hz)], fs_hz)[0]
    out = out[0] if a.ndim == 1 else out
    return _lib.to_host(out) if from_numpy else out


def ofdm_fft_used_batched(x, n_fft: int | None = None, bins=None) -> torch.Tensor:
    """ofdm_fft_used of every row of x[B, T] -> complex128 [B, n_used] on the device."""
    batch = _lib.as_batch(x, batched=True)
    if batch.nb != 1:
        raise ValueError("ofdm_fft_used_batched takes rows [B, T]")
    N = int(N_FFT if n_fft is None else n_fft)
    k = centered_subcarrier_indices(NUM_ACTIVE_SUBCARRIERS) if bins is None else np.asarray(bins)
    kb = torch.as_tensor(k.astype(np.int32)).to(batch.data.device)
    out = torch.empty((batch.B, k.size), dtype=torch.complex128, device=batch.data.device)
    _lib.check(_lib.lib().ofs_fft_used(batch.fmt, batch.data.data_ptr(), batch.B, batch.T, N, int(k.size),
                                       kb.data_ptr(), out.data_ptr(), _lib.stream_ptr()), "ofs_fft_used")
    return out


def ofdm_fft_used(symbol_time_no_cp):
    """FFT an OFDM symbol (no CP) and return only used, centered subcarriers (core.py:171-176);
    N_FFT and NUM_ACTIVE_SUBCARRIERS are read from this module at call time."""
    from_numpy = not isinstance(symbol_time_no_cp, torch.Tensor)
    a = np.asarray(symbol_time_no_cp) if from_numpy else symbol_time_no_cp
    if a.ndim != 1:
        raise ValueError("ofdm_fft_used takes one symbol (1-D samples)")
    out = ofdm_fft_used_batched(a[None])[0]
    return _lib.to_host(out) if from_numpy else out


def _cdiv(y, d, eps):
    dev = _lib.require_gpu()
    t, from_numpy, nd = _rows(y, dev)
    B, n = t.shape
    dn = d.dim() if isinstance(d, torch.Tensor) else np.ndim(d)
    if nd == 1 and dn == 2:                  # numpy broadcasting: a [n] numerator against [B, n] rows
        Bd = int(d.shape[0])
        t, B, nd = t.expand(Bd, n).contiguous(), Bd, 2
    r, rs = _ref_rows(d, B, n, dev)
    out = torch.empty_like(t)
    _lib.check(_lib.lib().ofs_cdiv_eps(t.data_ptr(), B, n, r.data_ptr(), rs, float(eps), out.data_ptr(),
                                       _lib.stream_ptr()), "ofs_cdiv_eps")
    return _out(out, from_numpy, nd)


def ls_channel_estimate(y_used, x_used, eps: float = 1e-9):
    """Least-squares per-subcarrier channel estimate H = Y / (X + eps) (core.py:339-341),
    numpy's complex division bit for bit.  [B, n] rows with a shared [n] X broadcast."""
    return _cdiv(y_used, x_used, eps)


def equalize(y_used, h_est, eps: float = 1e-9):
    """Y / (H + eps) (core.py:344-345), numpy's complex division bit for bit."""
    return _cdiv(y_used, h_est, eps)


def remove_common_phase(x, ref=None):
    """De-rotate by the common phase error (core.py:348-354): the angle of mean(x), or of
    vdot(ref, x) / (vdot(ref, ref) + 1e-12) when ref is given.  Returns (x * exp(-i cpe), cpe);
    for [B, n] rows cpe is a [B] array / tensor."""
    dev = _lib.require_gpu()
    t, from_numpy, nd = _rows(x, dev)
    B, n = t.shape
    if n == 0:                                          # np.mean of nothing: nan
        cpe = float("nan")
        return (np.array(x, dtype=np.complex128, copy=True) if from_numpy else x.clone()), cpe
    r, rs = _ref_rows(ref, B, n, dev) if ref is not None else (None, 0)
    out = torch.empty_like(t)
    cpe = torch.empty((B,), dtype=torch.float64, device=dev)
    _lib.check(_lib.lib().ofs_common_phase(t.data_ptr(), B, n, _lib.ptr(r), rs, out.data_ptr(), cpe.data_ptr(),
                                           _lib.stream_ptr()), "ofs_common_phase")
    c = float(cpe[0].item()) if nd == 1 else (_lib.to_host(cpe) if from_numpy else cpe)
    return _out(out, from_numpy, nd), c


def align_complex_gain(x, ref, eps: float = 1e-12):
    """Scale x by the complex gain g = vdot(x, ref) / (vdot(x, x) + eps) that best fits ref in
    the LS sense (core.py:357-362).  Returns (x * g, g)."""
    dev = _lib.require_gpu()
    t, from_numpy, nd = _rows(x, dev)
    B, n = t.shape
    r, rs = _ref_rows(ref, B, n, dev)
    out = torch.empty_like(t)
    g = torch.empty((B,), dtype=torch.complex128, device=dev)
    _lib.check(_lib.lib().ofs_align_gain(t.data_ptr(), B, n, r.data_ptr(), rs, float(eps), out.data_ptr(),
                                         g.data_ptr(), _lib.stream_ptr()), "ofs_align_gain")
    gg = complex(g[0].item()) if nd == 1 else (_lib.to_host(g) if from_numpy else g)
    return _out(out, from_numpy, nd), gg


def evm_rms_db(x, ref):
    """(evm_rms, evm_db), EVM normalised to the reference RMS magnitude (core.py:365-370)."""
    dev = _lib.require_gpu()
    t, from_numpy, nd = _rows(x, dev)
    B, n = t.shape
    r, rs = _ref_rows(ref, B, n, dev)
    evm = torch.empty((B,), dtype=torch.float64, device=dev)
    db = torch.empty((B,), dtype=torch.float64, device=dev)
    if n == 0:
        evm.fill_(float("nan"))
        db.fill_(float("nan"))
    else:
        _lib.check(_lib.lib().ofs_evm(t.data_ptr(), B, n, r.data_ptr(), rs, evm.data_ptr(), db.data_ptr(),
                                      _lib.stream_ptr()), "ofs_evm")
    if nd == 1:
        return float(evm[0].item()), float(db[0].item())
    return (_lib.to_host(evm), _lib.to_host(db)) if from_numpy else (evm, db)


def estimate_timing_offset_from_phase_slope(h_used):
    """Residual timing from the linear phase slope of an LS channel (core.py:443-469): unwrap
    angle(h) over the centred subcarriers of NUM_ACTIVE_SUBCARRIERS (read at call time), fit a
    line, return (slope_rad_per_bin, -slope * N_FFT / (2 pi)); (0.0, 0.0) for an empty h."""
    dev = _lib.require_gpu()
    t, from_numpy, nd = _rows(h_used, dev)
    B, n = t.shape
    if n == 0:
        return 0.0, 0.0
    k = centered_subcarrier_indices(NUM_ACTIVE_SUBCARRIERS)
    if k.size != n:
        raise ValueError(f"operands could not be broadcast together with shapes ({k.size},) ({n},)")
    kb = torch.as_tensor(k.astype(np.int32)).to(dev)
    slope = torch.empty((B,), dtype=torch.float64, device=dev)
    sto = torch.empty((B,), dtype=torch.float64, device=dev)
    _lib.check(_lib.lib().ofs_phase_slope(t.data_ptr(), B, n, kb.data_ptr(), int(N_FFT), slope.data_ptr(),
                                          sto.data_ptr(), _lib.stream_ptr()), "ofs_phase_slope")
    if nd == 1:
        return float(slope[0].item()), float(sto[0].item())
    return (_lib.to_host(slope), _lib.to_host(sto)) if from_numpy else (slope, sto)
