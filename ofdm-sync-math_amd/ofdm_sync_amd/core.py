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
