"""Synthetic receive-stream batches for benchmarks and tests (input synthesis, not the hot path).

Restates the reference's input builders (pinned to the reference's own outputs in
tests/test_host_logic.py against tests/golden/synth_builders.npz):
  aa_preamble      <- sync_aa.build_aa_preamble (sync_aa.py:160-235)
  load_cir         <- channel.load_measured_cir (channel.py:15-48)
  qpsk_symbol      <- sync_aa.build_random_qpsk_symbol (sync_aa.py:238-260), draws given
  frame            <- run_single_test's frame assembly (sync_aa.py:702-712)
  frames_batch     <- the whole run_single_test chain per stream on the GPU (ofs_synth_frames:
                      own QPSK payload per stream, CIR convolution, AWGN, CFO, 12-bit ADC)
  make_aa_batch    <- a cheaper form for the headline batch: one faded preamble (preamble ⊛ CIR)
  synth_batch         shifted per stream + CFO + AWGN (ofs_synth_batch).
Philox RNG on the GPU: distribution-level parity with numpy.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
CIR_DIR = os.path.join(_HERE, "channel_models")


def aa_preamble(total_length: int = 1024, n_fft: int = 1024, num_active: int = 600) -> np.ndarray:
    """[A][A] Zadoff-Chu preamble on every K-th bin (sync_aa.py:160-235)."""
    K = 2 * n_fft // total_length
    dc = n_fft // 2
    half_active = num_active // 2
    used = np.array([dc + o for o in range(-half_active, half_active + 1) if o != 0 and (dc + o) % K == 0])
    num_sc = len(used)
    root = 25 if num_sc % 25 != 0 else 23
    n = np.arange(num_sc)
    zc = np.exp(-1j * np.pi * root * n * (n + 1) / num_sc)
    spec = np.zeros(n_fft, complex)
    spec[used] = zc
    full = np.fft.ifft(spec) * np.sqrt(n_fft)
    pre = full[:total_length]
    return pre / np.sqrt(np.mean(np.abs(pre) ** 2))


def load_cir(name: str = "cir1") -> np.ndarray:
    """All RX-branch CIRs of a measured profile, [n_branch, taps] complex128."""
    data = np.genfromtxt(os.path.join(CIR_DIR, f"{name}.csv"), delimiter=",", skip_header=1)
    if data.ndim == 1:
        data = data[np.newaxis, :]
    chans = []
    for c in range((data.shape[1] - 1) // 2):
        re, im = data[:, 1 + 2 * c], data[:, 2 + 2 * c]
        m = np.isfinite(re) & np.isfinite(im)
        chans.append(re[m] + 1j * im[m])
    out = np.zeros((len(chans), max(len(c) for c in chans)), complex)
    for i, c in enumerate(chans):
        out[i, :len(c)] = c
    return out


# frame geometry of sync_aa.run_single_test (sync_aa.py:99-125, :699-712)
N_FFT = 1024
CYCLIC_PREFIX = 72
NUM_ACTIVE = 600
PRE_PAD = 500
POST_PAD = 500


def active_bins(n_fft: int = N_FFT, num_active: int = NUM_ACTIVE) -> np.ndarray:
    """FFT bins of the centred active subcarriers after ifftshift (sync_aa.py:131-145 + the
    ifftshift of :247): centred index k -> bin k mod N."""
    half = num_active // 2
    k = np.concatenate([np.arange(-half, 0), np.arange(1, half + 1)])
    return (k % n_fft).astype(np.int32)


def qpsk_symbol(phases, n_fft: int = N_FFT, cp: int = CYCLIC_PREFIX) -> np.ndarray:
    """Random-QPSK OFDM symbol with CP from its phase indices (0..3 per active subcarrier):
    restates sync_aa.build_random_qpsk_symbol (sync_aa.py:238-260) with the draws given."""
    phases = np.asarray(phases)
    q = np.exp(1j * np.pi / 4 * (2 * phases + 1)) / np.sqrt(2)
    spec = np.zeros(n_fft, complex)
    spec[active_bins(n_fft, len(phases))] = q
    sym = np.fft.ifft(spec) * np.sqrt(n_fft)
    sym = sym / np.sqrt(np.mean(np.abs(sym) ** 2))
    return np.concatenate([sym[-cp:], sym])


def frame(preamble, symbols, pre_pad: int = PRE_PAD, post_pad: int = POST_PAD) -> np.ndarray:
    """[pad][preamble][symbols...][pad] (sync_aa.py:705-712)."""
    return np.concatenate([np.zeros(pre_pad, complex), preamble, *symbols, np.zeros(post_pad, complex)])


def faded_base(L: int = 512, cir: str | None = "cir1", branches=(1,)) -> np.ndarray:
    """[n_branch, len] unit-power faded [A][A] preamble (preamble ⊛ CIR of each branch), the
    deterministic part of every synthesised stream."""
    pre = aa_preamble(2 * L)
    rows = []
    for br in branches:
        y0 = pre if cir is None else np.convolve(pre, load_cir(cir)[br])
        rows.append(y0 / np.sqrt(np.mean(np.abs(y0[: 2 * L]) ** 2)))
    n = max(len(r) for r in rows)
    out = np.zeros((len(rows), n), complex)
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out


_FMT = {torch.complex64: _lib.C64, torch.complex128: _lib.C128, torch.int16: _lib.CI16}


def synth_batch(base, B: int, T: int, *, max_offset: int = 128, snr_db=(0.0, 15.0), cfo_hz=(-5000.0, 5000.0),
                fs: float = 15.36e6, seed: int = 2026, device="cuda", dtype=torch.complex64,
                adc_scale: float = 1024.0, return_params: bool = False):
    """ofs_synth_batch: [B, n_branch, T] streams = base shifted by a random offset, CFO tone,
    AWGN at a random SNR (per stream), optionally int12-quantised (dtype=torch.int16 -> I/Q
    pairs in a trailing axis).  Generated on the GPU in one kernel."""
    base = np.atleast_2d(np.asarray(base, np.complex128))
    nb, Lb = base.shape
    dev = torch.device(device)
    bt = torch.from_numpy(np.ascontiguousarray(base)).to(dev)
    if dtype not in _FMT:
        raise TypeError(f"unsupported output dtype {dtype}")
    shape = (B, nb, T, 2) if dtype == torch.int16 else (B, nb, T)
    out = torch.empty(shape, dtype=dtype, device=dev)
    params = torch.empty((B, 3), dtype=torch.float64, device=dev) if return_params else None
    with torch.cuda.device(dev):
        rc = _lib.lib().ofs_synth_batch(bt.data_ptr(), Lb, nb, B, T, int(max_offset), float(snr_db[0]),
                                        float(snr_db[1]), float(cfo_hz[0]), float(cfo_hz[1]), float(fs),
                                        int(seed) & ((1 << 64) - 1), _FMT[dtype], float(adc_scale), out.data_ptr(),
                                        _lib.ptr(params), torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(rc, "ofs_synth_batch")
    torch.cuda.current_stream(dev).synchronize()           # `bt` is freed on return
    return (out, params) if return_params else out


def make_aa_batch(B: int, T: int = 1024, L: int = 512, *, seed: int = 2026, cir: str | None = "cir1",
                  branch: int = 1, snr_db=(0.0, 15.0), cfo_hz=(-5000.0, 5000.0), fs: float = 15.36e6,
                  max_offset: int = 128, device="cuda", dtype=torch.complex64) -> torch.Tensor:
    """Batch [B, 1, T] of received [A][A] preambles: CIR (one branch) + AWGN + CFO, unit power.

    Each stream is a T-sample window of the faded preamble starting at a random offset in
    [0, max_offset); SNR and CFO are drawn uniformly per stream (ofs_synth_batch on the GPU).
    """
    return synth_batch(faded_base(L, cir, (branch,)), B, T, max_offset=max_offset, snr_db=snr_db, cfo_hz=cfo_hz,
                       fs=fs, seed=seed, device=device, dtype=dtype)


class Frames:
    """Result of ``frames_batch``: x [B, n_br, T] (or [..., 2] int16 codes), params [B, 4] f64
    (window start, snr_db, cfo_hz, full scale), phases [B, n_sym, n_bins] u8 (QPSK draws)."""

    def __init__(self, x, params, phases, preamble, cir):
        self.x, self.params, self.phases, self.preamble, self.cir = x, params, phases, preamble, cir


def frames_batch(B: int, T: int | None = None, *, preamble_len: int = 1024, cir: str | None = "cir1",
                 n_br: int = 2, branches=None, n_sym: int = 2, snr_db=(0.0, 15.0), cfo_hz=(-5000.0, 5000.0),
                 fs: float = 15.36e6, full_scale_ratio: float | None = None, win_start: int = 0,
                 max_offset: int = 1, seed: int = 2026, device="cuda", dtype=torch.complex64,
                 return_phases: bool = False) -> Frames:
    """ofs_synth_frames: B independent frames of sync_aa.run_single_test (sync_aa.py:699-738) -
    [A][A] preamble + n_sym random-QPSK symbols (per stream) between 500-sample pads, per-branch
    CIR convolution, AWGN at a per-stream SNR, CFO, optional 12-bit ADC (full_scale_ratio) -
    generated on the GPU.  T defaults to the whole received frame (pads + preamble + symbols +
    taps - 1); the window starts at win_start + U{0..max_offset-1}.  cir None: AWGN only
    (a one-tap identity channel, as apply_channel_multi_antenna's channel_name=None).
    ``branches``: CIR bank rows to use (default the first n_br, as the reference)."""
    pre = aa_preamble(preamble_len)
    if cir is None:
        h = np.ones((n_br, 1), complex)
    elif branches is not None:
        h = load_cir(cir)[list(branches)]
        n_br = h.shape[0]
    else:
        h = load_cir(cir)[:n_br]
        if h.shape[0] < n_br:                                 # sync_aa.py:603-606: tile the bank
            h = np.tile(h, (n_br // h.shape[0] + 1, 1))[:n_br]
    pc = np.stack([np.convolve(pre, h[br]) for br in range(n_br)])
    bins = active_bins()
    Lout = PRE_PAD + preamble_len + n_sym * (N_FFT + CYCLIC_PREFIX) + POST_PAD + h.shape[1] - 1
    T = Lout if T is None else int(T)
    dev = torch.device(device)
    if dtype not in _FMT:
        raise TypeError(f"unsupported output dtype {dtype}")
    shape = (B, n_br, T, 2) if dtype == torch.int16 else (B, n_br, T)
    out = torch.empty(shape, dtype=dtype, device=dev)
    params = torch.empty((B, 4), dtype=torch.float64, device=dev)
    phases = torch.empty((B, n_sym, len(bins)), dtype=torch.uint8, device=dev) if return_phases else None
    pct = torch.from_numpy(np.ascontiguousarray(pc)).to(dev)
    ht = torch.from_numpy(np.ascontiguousarray(h.astype(np.complex128))).to(dev)
    bt = torch.from_numpy(bins).to(dev)
    with torch.cuda.device(dev):
        rc = _lib.lib().ofs_synth_frames(pct.data_ptr(), pc.shape[1], ht.data_ptr(), h.shape[1], n_br, PRE_PAD,
                                         preamble_len, n_sym, N_FFT, CYCLIC_PREFIX, bt.data_ptr(), len(bins),
                                         POST_PAD, B, T, int(win_start), int(max_offset), float(snr_db[0]),
                                         float(snr_db[1]), float(cfo_hz[0]), float(cfo_hz[1]), float(fs),
                                         float(full_scale_ratio or 0.0), int(seed) & ((1 << 64) - 1), _FMT[dtype],
                                         out.data_ptr(), params.data_ptr(), _lib.ptr(phases),
                                         torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(rc, "ofs_synth_frames")
    torch.cuda.current_stream(dev).synchronize()             # host-built inputs are freed on return
    return Frames(out, params, phases, pre, h)


def headline_batch(B: int, T: int = 1024, L: int = 512, *, seed: int = 2026, device="cuda",
                   dtype=torch.complex64) -> torch.Tensor:
    """The bench's cfg3 input: [B, 1, T] windows of per-stream run_single_test frames
    ([A][A] preamble of 2L, own QPSK payload, cir1 RX branch 1, AWGN U[0, 15] dB, CFO U[-5, 5] kHz
    at 15.36 MHz), each window starting U{0..127} samples before the preamble + 64."""
    return frames_batch(B, T, preamble_len=2 * L, cir="cir1", branches=(1,), snr_db=(0.0, 15.0),
                        cfo_hz=(-5000.0, 5000.0), win_start=PRE_PAD - 64, max_offset=128, seed=seed,
                        device=device, dtype=dtype).x


def make_aa_batch_torch(B: int, T: int = 1024, L: int = 512, *, seed: int = 2026, cir: str | None = "cir1",
                        branch: int = 1, snr_db=(0.0, 15.0), cfo_hz=(-5000.0, 5000.0), fs: float = 15.36e6,
                        max_offset: int = 128, device="cuda", dtype=torch.complex64) -> torch.Tensor:
    """make_aa_batch with torch ops on any device (CPU included): the input generator of the
    CPU-only multi-process tests (gloo), where the HIP kernel cannot run.  Same distribution,
    different random stream.

    Each stream is a T-sample window of the faded preamble starting at a random offset in
    [0, max_offset); SNR and CFO are drawn uniformly per stream.
    """
    rng = np.random.default_rng(seed)
    pre = aa_preamble(2 * L)
    y0 = pre if cir is None else np.convolve(pre, load_cir(cir)[branch])
    y0 = y0 / np.sqrt(np.mean(np.abs(y0[: 2 * L]) ** 2))
    pad = np.zeros(T + max_offset, complex)
    pad[: min(len(y0), len(pad))] = y0[: len(pad)]
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    base = torch.from_numpy(pad).to(dev)
    off = torch.from_numpy(rng.integers(0, max_offset, B)).to(dev)
    idx = off[:, None] + torch.arange(T, device=dev)[None, :]
    sig = base[idx]                                                        # [B, T] c128
    snr = torch.from_numpy(rng.uniform(*snr_db, B)).to(dev)
    f = torch.from_numpy(rng.uniform(*cfo_hz, B)).to(dev)
    nstd = torch.sqrt(10 ** (-snr / 10) / 2)[:, None]
    noise = torch.complex(torch.randn((B, T), generator=g, device=dev, dtype=torch.float64),
                          torch.randn((B, T), generator=g, device=dev, dtype=torch.float64)) * nstd
    n = torch.arange(T, device=dev, dtype=torch.float64)
    tone = torch.polar(torch.ones((B, T), device=dev, dtype=torch.float64), 2 * np.pi * f[:, None] * n[None, :] / fs)
    x = (sig * tone + noise).to(dtype)
    return x[:, None, :].contiguous()
