"""Integer-exact wave-per-stream kernels (csrc/aa_exact.hip) for int16 I/Q input.

For int16 samples every product and window sum is an exact integer, so the exact kernels and
the general LDS engine (forced with variant EXACT=0) must agree BIT FOR BIT although they sum in
different orders: P, R, M, valid and the events of sync_aa (sync_aa.py:421-571); all eight
arrays and the gate events of minn_rtl (minn_rtl.py:583-825).  Integer arrays are also checked
against the CPU oracle (bit-exact), which is itself pinned to the reference's goldens.
"""
from __future__ import annotations

import numpy as np
import pytest

import ofdm_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from ofdm_sync_amd import _lib, minn_rtl, sync_aa  # noqa: E402

RTL_KEYS = ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled",
            "energy_scaled", "metric_valid", "above_threshold")


def _int12_bursts(rng, B, nb, T, blocks, amp=1500, noise=60):
    """int16 I/Q [B, nb, T, 2]: int12 noise plus, in every other stream, a burst made of the
    given block pattern (e.g. [1, 1] for [A][A], [1, 1, -1, -1] for Minn) of a random segment."""
    x = rng.normal(0, noise, (B, nb, T)) + 1j * rng.normal(0, noise, (B, nb, T))
    seg = len(blocks[1])
    for b in range(0, B, 2):
        n = seg * len(blocks[0])
        if T > n + 2:
            s = int(rng.integers(0, T - n))
            a = rng.normal(0, amp / 3, seg) + 1j * rng.normal(0, amp / 3, seg)
            burst = np.concatenate([sgn * a for sgn in blocks[0]])
            x[b, :, s:s + n] += burst
    re = np.clip(np.round(x.real), -2048, 2047)
    im = np.clip(np.round(x.imag), -2048, 2047)
    return np.stack([re, im], axis=-1).astype(np.int16)


def _aa_run(xt, L, variant, exact: bool):
    variant("EXACT", 1 if exact else 0)
    out = sync_aa.aa_detect_streaming_batched(xt, L=L, threshold=0.15, hysteresis=16)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("B,nb,T,L", [(37, 1, 1024, 128), (9, 2, 999, 256), (5, 1, 5000, 512),
                                      (6, 2, 700, 64), (3, 1, 2300, 1024)])
def test_aa_exact_kernel_bit_identical_to_general_engine(B, nb, T, L, variant):
    rng = np.random.default_rng(B * 7 + L)
    iq = _int12_bursts(rng, B, nb, T, ([1, 1], np.zeros(L)))
    xt = torch.from_numpy(iq).cuda()
    plan = _lib.lib().ofs_aa_plan(_lib.CI16, _lib.FP64, nb, T, L)
    assert 2000 < plan < 3000, plan                    # the exact kernel serves this shape
    a = _aa_run(xt, L, variant, True)
    g = _aa_run(xt, L, variant, False)
    for k in ("P", "R", "M", "valid", "n_events"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    n = a.n_events.cpu().numpy()
    assert n[::2].sum() > 0                            # bursts open gates
    for b in range(B):
        assert torch.equal(a.ev_int[b, :n[b]], g.ev_int[b, :n[b]])
        assert torch.equal(a.ev_real[b, :n[b]], g.ev_real[b, :n[b]])
    for b in (0, B - 1):                               # and the oracle (integer P, R exact)
        xc = (iq[b, ..., 0] + 1j * iq[b, ..., 1]).astype(np.complex128)
        P, R, M, v = O.aa_metric(xc, L)
        assert np.array_equal(a.P[b].cpu().numpy(), P)
        assert np.array_equal(a.R[b].cpu().numpy(), R)
        assert np.max(np.abs(a.M[b].cpu().numpy() - M)) < 1e-12
        assert np.array_equal(a.valid[b].cpu().numpy(), v)


def _rtl_run(xt, Q, variant, exact, **kw):
    variant("EXACT", 1 if exact else 0)
    out = minn_rtl.minn_rtl_batched(xt, Q, **kw)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("B,nb,T,Q", [(33, 1, 1024, 64), (7, 2, 777, 64), (5, 3, 3000, 128),
                                      (4, 1, 4096, 512), (6, 2, 2500, 256)])
@pytest.mark.parametrize("mode,shift,hyst", [("float", 3, 2), ("floor", 3, 2), ("float", 0, 0), ("floor", 0, 1), ("floor", 6, 3)])
def test_rtl_exact_kernel_bit_identical_to_general_engine(B, nb, T, Q, mode, shift, hyst, variant):
    rng = np.random.default_rng(B + Q + shift)
    iq = _int12_bursts(rng, B, nb, T, ([1, 1, -1, -1], np.zeros(Q)))
    xt = torch.from_numpy(iq).cuda()
    assert _lib.lib().ofs_rtl_plan(_lib.CI16, nb, T, Q) > 2000
    kw = dict(smooth_shift=shift, threshold_value=3276, threshold_frac_bits=15, smooth_mode=mode,
              hysteresis=hyst, timing_offset=-5)
    a = _rtl_run(xt, Q, variant, True, **kw)
    g = _rtl_run(xt, Q, variant, False, **kw)
    for k in RTL_KEYS + ("n_events", "open_gate_start"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    n = a.n_events.cpu().numpy()
    assert n.sum() > 0
    for b in range(B):
        m = min(int(n[b]), a.events.shape[1])
        assert torch.equal(a.events[b, :m], g.events[b, :m])
    xc = (iq[0, ..., 0] + 1j * iq[0, ..., 1]).astype(np.complex128)
    s = O.minn_rtl_metric(xc, Q, shift, 3276, 15, smooth_mode=mode)
    for k in RTL_KEYS:
        assert np.array_equal(getattr(a, k)[0].cpu().numpy(), s[k]), k
    ev, _, _ = O.detect_minn_rtl(s["corr_positive"], s["above_threshold"], s["metric_valid"], hyst, -5)
    assert np.array_equal(a.events[0, :int(n[0])].cpu().numpy(), ev)


def test_rtl_exact_metric_only_outputs():
    """Metric without smoothing outputs or gate (the optional arrays of ofs_minn_rtl are null
    except corr_total / energy_total): exact kernel skips the sequential pass."""
    rng = np.random.default_rng(3)
    iq = _int12_bursts(rng, 4, 1, 1024, ([1, 1, -1, -1], np.zeros(64)))
    xt = torch.from_numpy(iq).cuda()
    B, T = 4, 1024
    ct = torch.empty((B, T), dtype=torch.float64, device="cuda")
    et = torch.empty_like(ct)
    rc = _lib.lib().ofs_minn_rtl(_lib.CI16, xt.data_ptr(), B, 1, T, 64, 3, 0, 3276, 15, ct.data_ptr(),
                                 None, None, et.data_ptr(), None, None, None, None, 0, 0, 0, 0, None,
                                 None, None, _lib.stream_ptr())
    assert rc == 0
    ref = minn_rtl.minn_rtl_batched(xt, 64, detect=False)
    assert torch.equal(ct, ref.corr_total) and torch.equal(et, ref.energy_total)


def test_exact_plans_fall_back_outside_exact_range():
    L_ = _lib.lib()
    assert L_.ofs_aa_plan(_lib.CI16, _lib.FP64, 1, 1024, 192) < 2000          # L not covered
    assert not 2000 < L_.ofs_aa_plan(_lib.C128, _lib.FP64, 1, 1024, 128) < 3000  # float input: not integer-exact
    assert L_.ofs_aa_plan(_lib.CI16, _lib.FP64, 1, (1 << 21) + 2, 128) < 2000  # sums may pass 2^53
    assert L_.ofs_rtl_plan(_lib.CI16, 1, 1024, 1024) == 0                     # Q > 512
    assert L_.ofs_rtl_plan(_lib.C128, 1, 1024, 64) == 0


@pytest.mark.parametrize("shift", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("T", [1024, 2100, 513])
def test_rtl_segment_parallel_iir_is_exact(shift, T, variant):
    """The segment-parallel IIR (aa_exact.hip: guessed chunk states, exact chunk runs iterated
    to a self-consistent chain) equals the general engine's sequential recursion and the
    oracle bit for bit, across contraction factors and partial segments."""
    rng = np.random.default_rng(100 + shift + T)
    B, nb, Q = 9, 2, 64
    iq = _int12_bursts(rng, B, nb, T, ([1, 1, -1, -1], np.zeros(Q)))
    xt = torch.from_numpy(iq).cuda()
    kw = dict(smooth_shift=shift, threshold_value=3276, threshold_frac_bits=15, smooth_mode="float",
              hysteresis=2, timing_offset=0)
    a = _rtl_run(xt, Q, variant, True, **kw)
    g = _rtl_run(xt, Q, variant, False, **kw)
    for k in RTL_KEYS + ("n_events", "open_gate_start"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    xc = (iq[1, ..., 0] + 1j * iq[1, ..., 1]).astype(np.complex128)
    s = O.minn_rtl_metric(xc, Q, shift, 3276, 15)
    for k in RTL_KEYS:
        assert np.array_equal(getattr(a, k)[1].cpu().numpy(), s[k]), k


def _rtl_check_every_stream(iq, Q, variant, shift, hyst=2, toff=0, mode="float"):
    """Exact kernel vs the general engine (EXACT=0, sequential recursion) AND the C oracle
    (oracle_c.minn_rtl: minn_rtl.py:583-825 restated statement for statement) on EVERY stream,
    every array bit for bit, every event."""
    import oracle_c
    xt = torch.from_numpy(iq).cuda()
    kw = dict(smooth_shift=shift, threshold_value=3276, threshold_frac_bits=15, smooth_mode=mode,
              hysteresis=hyst, timing_offset=toff)
    a = _rtl_run(xt, Q, variant, True, **kw)
    g = _rtl_run(xt, Q, variant, False, **kw)
    for k in RTL_KEYS + ("n_events", "open_gate_start"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    n = a.n_events.cpu().numpy()
    for b in range(iq.shape[0]):
        m = min(int(n[b]), a.events.shape[1])
        assert torch.equal(a.events[b, :m], g.events[b, :m]), b
    if mode != "float":
        return a
    xc = (iq[..., 0] + 1j * iq[..., 1]).astype(np.complex128)
    o = oracle_c.minn_rtl(xc, Q, shift, 3276, 15, hyst, toff, max_events=int(a.events.shape[1]), nthreads=8)
    for k in ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled", "energy_scaled"):
        assert np.array_equal(getattr(a, k).cpu().numpy(), o[k]), k
    assert np.array_equal(a.metric_valid.cpu().numpy(), o["metric_valid"].astype(bool))
    assert np.array_equal(a.above_threshold.cpu().numpy(), o["above_threshold"].astype(bool))
    assert np.array_equal(n, o["n_events"])
    ev = a.events.cpu().numpy()
    for b in range(iq.shape[0]):
        k = min(int(n[b]), ev.shape[1])
        assert np.array_equal(ev[b, :k], o["events"][b, :k]), b
    return a


@pytest.mark.parametrize("shift", [9, 12, 14, 15])
@pytest.mark.parametrize("T", [1024, 2100, 4096])
def test_rtl_fast_iir_slow_contraction_every_stream(shift, T, variant):
    """Shifts 9-14 take the fma fast path of the segment-parallel IIR (aa_exact.hip, `interior`),
    where the speculation chain contracts slowest per chunk (keep = 1 - 2^-shift) and needs the most
    rounds; 15 is the first shift past it (the per-sample-select path).  minn_rtl.py:704-722."""
    rng = np.random.default_rng(1000 + 7 * shift + T)
    B, nb, Q = 12, 2, 64
    iq = _int12_bursts(rng, B, nb, T, ([1, 1, -1, -1], np.zeros(Q)))
    a = _rtl_check_every_stream(iq, Q, variant, shift)
    sm = a.smooth_metric.cpu().numpy()
    assert (sm[:, -1] > 0).all()                       # the state is live through every segment


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_rtl_fast_iir_long_decay_through_guard(shift, variant):
    """A burst followed by an all-zero tail: corr_positive is exactly 0 after the window passes,
    so the IIR state decays by (1 - 2^-shift) per sample through the 2^-700 guard of the fast path
    (aa_exact.hip `fast`) into the subnormal range and to 0.  Every stream bit for bit."""
    rng = np.random.default_rng(40 + shift)
    B, nb, Q, T = 8, 1, 64, 8192
    x = np.zeros((B, nb, T), np.complex128)
    for b in range(B):
        s = int(rng.integers(0, 300))
        blk = rng.normal(0, 500, Q) + 1j * rng.normal(0, 500, Q)
        x[b, 0, :s] = rng.normal(0, 40, s) + 1j * rng.normal(0, 40, s)
        x[b, 0, s:s + 4 * Q] = np.concatenate([blk, blk, -blk, -blk])
    re = np.clip(np.round(x.real), -2048, 2047)
    im = np.clip(np.round(x.imag), -2048, 2047)
    iq = np.stack([re, im], axis=-1).astype(np.int16)
    a = _rtl_check_every_stream(iq, Q, variant, shift)
    sm = a.smooth_metric.cpu().numpy()
    tiny = (sm > 0) & (sm < 2.0 ** -700)
    assert tiny.any(axis=1).all()                      # every stream passes below the guard
    assert (sm[:, -1] < 2.0 ** -1000).all()               # into the subnormal range


@pytest.mark.parametrize("nb,Q", [(1, 64), (1, 256), (2, 64), (2, 256), (1, 128)])
def test_rtl_exact_full_range_int16_after_int12_rows(nb, Q, variant):
    """int16 words beyond 12 bits (+-30000) arriving after rows of 12-bit words: the int32 row-scan
    path (aa_exact.hip IROW, nb = 1, E = 1 / 2) must switch to the fp64 scan at the first wide row
    and carry the integer prefix across the switch.  Every stream bit for bit vs EXACT=0 and the
    C oracle, in both IIR modes."""
    rng = np.random.default_rng(500 + nb * Q)
    B, T = 10, 3000
    iq = _int12_bursts(rng, B, nb, T, ([1, 1, -1, -1], np.zeros(Q))).astype(np.int32)
    for b in range(B):
        s = 64 * int(rng.integers(1, 20)) + int(rng.integers(0, 64)) * (b % 2)   # wide from some row on
        n = int(rng.integers(8, 600))
        iq[b, :, s:s + n] = rng.integers(-30000, 30001, (nb, n, 2))
        if b % 3 == 0:
            iq[b, :, s + n + 500:] = rng.choice([-32768, 32767], (nb, T - s - n - 500, 2)) if T > s + n + 500 else 0
    iq = iq.astype(np.int16)
    _rtl_check_every_stream(iq, Q, variant, 3)
    _rtl_check_every_stream(iq, Q, variant, 3, mode="floor")
