"""GPU parity for the correlation-shaped metrics (csrc/corr.hip), through the C ABI:
Park (park.py:64-114), the ZC frequency-domain metric (zc_freq.py:62-99), the ZC matched
filter / normaliser / combiner (zc_v2.py:244-271, zc.py:106-126) and the zc_v2 CFAR + gate
(zc_v2.py:300-446), against the reference goldens and the CPU oracle.

Tolerances (written here):
  fp64 paths: complex sums within 1e-11 of the stream maximum; normalised metrics within
      1e-9 relative + 1e-11 absolute (a direct O(N) sum or a sliding DFT in a different
      summation order than numpy's pocketfft / np.convolve);
  fp32 Park (complex64 input) and fp32 zc_freq (window FFT): every output within the fp32 error
      models of tests/error_models.py (models 3 and 2), measured ratio printed;
  CFAR/gate given the same corr_mag: bit-identical (the kernel runs the reference's
      sequential float64 recursion); end to end, events identical and flags identical
      except at samples whose threshold margin is below 1e-9 relative.
"""
import os

import numpy as np
import pytest

import error_models as EM
import ofdm_oracle as O
import oracle_c
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import park, zc_freq, zc_v2, zc  # noqa: E402


def G(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b)) / max(1e-300, float(np.max(np.abs(b)))))


def rng_c(rng, *shape):
    return rng.standard_normal(shape) + 1j * rng.standard_normal(shape)


# ------------------------------------------------------------------ Park ---------------
@pytest.mark.parametrize("name", ["park_N2048", "park_N256", "park_N64"])
def test_park_vs_reference_golden(name, monkeypatch):
    d = G(name)
    monkeypatch.setattr(park, "N_FFT", int(d["N"]))
    ds, M, P, E = park.park_streaming_metric(d["x"])
    assert isinstance(M, np.ndarray) and M.dtype == np.float64 and P.dtype == np.complex128
    assert np.array_equal(ds, d["ds"])
    assert rel(P, d["P"]) < 1e-11
    assert rel(E, d["E"]) < 1e-12
    np.testing.assert_allclose(M, d["M"], rtol=1e-9, atol=1e-11)
    assert int(np.argmax(M)) == int(np.argmax(d["M"]))


@pytest.mark.parametrize("N,T,nb,fmt", [(64, 400, 1, "c128"), (130, 1000, 2, "c128"), (65, 300, 3, "c128"),
                                        (512, 5000, 2, "i16"), (2048, 4097, 1, "c128"),
                                        (4096, 9000, 1, "c128"), (16, 17, 1, "c128")])
def test_park_batched_vs_oracle(N, T, nb, fmt):
    rng = np.random.default_rng(N + T)
    B = 3
    if fmt == "i16":
        xi = rng.integers(-2048, 2048, size=(B, nb, T, 2)).astype(np.int16)
        x = xi[..., 0] + 1j * xi[..., 1]
        ds, M, P, E = park.park_streaming_metric_batched(torch.from_numpy(xi).cuda(), N=N)
    else:
        x = rng_c(rng, B, nb, T)
        ds, M, P, E = park.park_streaming_metric_batched(torch.from_numpy(x).cuda(), N=N)
    for b in range(B):
        dso, Mo, Po, Eo = O.park_metric(x[b], N)
        assert np.array_equal(ds.cpu().numpy(), dso)
        assert rel(P[b].cpu().numpy(), Po) < 1e-11
        assert rel(E[b].cpu().numpy(), Eo) < 1e-12
        np.testing.assert_allclose(M[b].cpu().numpy(), Mo, rtol=1e-9, atol=1e-12)
        if fmt == "i16":                     # integer input: every partial sum exact
            assert np.array_equal(P[b].cpu().numpy(), Po) and np.array_equal(E[b].cpu().numpy(), Eo)


@pytest.mark.parametrize("N,nb", [(512, 1), (2048, 1), (256, 2)])
def test_park_fp32_complex64(N, nb):
    """fp32 Park within error model 3 (one fp32 FMA chain per output): |dP| <= sqrt(2)(2h·nb+2)u·S_abs,
    |dE| <= (2h·nb+10)u·E, M by first-order propagation; a stream with a 60 dB step included."""
    rng = np.random.default_rng(5 + N)
    x = rng_c(rng, 4, nb, 3000 + N).astype(np.complex64)
    x[2, :, 1500:] *= 1e-3
    ds, M, P, E = park.park_streaming_metric_batched(torch.from_numpy(x).cuda(), N=N)
    assert M.dtype == torch.float32
    worst = 0.0
    for b in range(4):
        xb = x[b].astype(np.complex128)
        _, Mo, Po, Eo = O.park_metric(xb, N)
        bP, bE = EM.park_bounds(xb, N)
        bM = EM.metric_bound(np.abs(Po), Eo, Mo, bP, bE)
        r = [np.max(np.abs(P[b].cpu().numpy().astype(np.complex128) - Po) / bP),
             np.max(np.abs(E[b].cpu().numpy().astype(np.float64) - Eo) / bE),
             np.max(np.abs(M[b].cpu().numpy().astype(np.float64) - Mo) / bM)]
        assert max(r) <= 1.0, r
        worst = max(worst, *r)
    print(f"park fp32 N={N} nb={nb}: max |err|/bound = {worst:.3g}")


def test_park_empty_like_reference(monkeypatch):
    monkeypatch.setattr(park, "N_FFT", 64)
    ds, M, P, E = park.park_streaming_metric(np.ones(64, complex))      # T < N+1
    assert ds.size == M.size == P.size == E.size == 0
    ds, M, P, E = park.park_streaming_metric(np.ones(65, complex))      # exactly one output
    assert list(ds) == [32] and M.size == 1


# ------------------------------------------------------------------ zc_freq ------------
@pytest.mark.parametrize("name", ["zcfreq_N2048", "zcfreq_N256"])
def test_zc_freq_vs_reference_golden(name, monkeypatch):
    d = G(name)
    monkeypatch.setattr(zc_freq, "N_FFT", int(d["N"]))
    monkeypatch.setattr(zc_freq, "CYCLIC_PREFIX", int(d["CP"]))
    idx, t, e = zc_freq.make_pss_frequency_template()
    assert np.array_equal(idx, d["bins"]) and e == float(d["template_energy"])
    m = zc_freq.compute_frequency_metric(d["x"], idx, t, e)
    assert m.dtype == np.float64 and m.shape == d["metric"].shape
    np.testing.assert_allclose(m, d["metric"], rtol=1e-9, atol=1e-11)
    assert int(np.argmax(m)) == int(np.argmax(d["metric"]))


@pytest.mark.parametrize("N,cp,T,nb", [(256, 64, 2000, 1), (256, 64, 2000, 2), (128, 0, 700, 3),
                                       (512, 128, 4000, 4), (4096, 1024, 6000, 1), (64, 16, 80, 1)])
def test_zc_freq_batched_vs_oracle(N, cp, T, nb):
    rng = np.random.default_rng(N * 7 + nb)
    B = 3
    x = rng_c(rng, B, nb, T)
    # a ZC-bearing symbol in stream 1 so the metric has a real peak
    idx, t, e = O.zc_template()
    if T >= 300 + N:
        x[1, :, 300:300 + N] += 4 * O.pss_symbol(N)
    m = zc_freq.compute_frequency_metric_batched(torch.from_numpy(x).cuda(), idx, t, e, N=N, cp=cp)
    for b in range(B):
        mo = O.zc_freq_metric(x[b], N, cp, idx, t, e)
        np.testing.assert_allclose(m[b].cpu().numpy(), mo, rtol=1e-9, atol=1e-11)


def test_zc_freq_too_short_raises(monkeypatch):
    monkeypatch.setattr(zc_freq, "N_FFT", 64)
    monkeypatch.setattr(zc_freq, "CYCLIC_PREFIX", 16)
    idx, t, e = zc_freq.make_pss_frequency_template()
    with pytest.raises(ValueError):
        zc_freq.compute_frequency_metric(np.ones(79, complex), idx, t, e)
    assert zc_freq.compute_frequency_metric(np.ones(80, complex), idx, t, e).shape == (1,)


# ------------------------------------------------------------------ ZC matched filter --
def test_zc_matched_filter_vs_reference_golden():
    d = G("zc_mf")
    x, ref = d["x"], d["ref"]
    for b in range(x.shape[0]):
        c = zc_v2.matched_filter_correlation(x[b], ref)
        assert c.dtype == np.complex128 and c.shape == d["corr"][b].shape
        assert rel(c, d["corr"][b]) < 1e-11
        nrm = zc_v2.normalize_correlation(d["corr"][b], x[b], ref)
        assert rel(nrm, d["norm"][b]) < 1e-11
    comb = zc.combined_matched_filter(x, d["zc_ref"])
    assert rel(comb, d["zc_combined"]) < 1e-11


def test_zc_detect_preamble_vs_reference_golden():
    d = G("zc_mf")
    r = zc_v2.detect_zc_preamble(d["x"])
    st = r.state
    np.testing.assert_allclose(st.corr_mag, d["corr_mag"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(st.local_sum, d["local_sum"], rtol=1e-9, atol=1e-9)
    assert np.array_equal(st.metric_valid, d["metric_valid"])
    # flags may only differ where the comparison margin is at rounding level
    diff = st.above_threshold != d["above_threshold"]
    margin = np.abs(d["corr_scaled"] - d["thresh_scaled"]) / np.maximum(np.abs(d["thresh_scaled"]), 1e-300)
    margin2 = np.abs(d["corr_mag"] - float(d["min_corr_mag"]))
    assert np.all((margin[diff] < 1e-9) | (margin2[diff] < 1e-9))
    ev = np.array([[e.peak_index, e.gate_start, e.gate_end, e.detected_start] for e in r.events]).reshape(-1, 4)
    assert np.array_equal(ev, d["events"])
    np.testing.assert_allclose([e.peak_value for e in r.events], d["peak_values"], rtol=1e-9)
    assert np.array_equal(r.gate_mask, d["gate_mask"])


@pytest.mark.parametrize("hyst,B,n,W", [(0, 4, 3000, 128), (1, 4, 3000, 128), (5, 4, 3000, 128), (64, 4, 3000, 128),
                                         (64, 11, 4096, 256), (100, 9, 2048, 128), (64, 5, 1536, 512),
                                         (256, 37, 2048, 256), (256, 20, 4096, 1024)])
def test_zc_cfar_and_gate_bit_identical_given_corr_mag(hyst, B, n, W):
    """CFAR + gate vs the oracle, bit for bit: the sequential kernel (hysteresis < 64), the fused
    lane-per-stream kernel with register-staged tiles (n not a whole number of chunks) and with
    LDS-DMA tiles (n and W whole chunks; 11, 9, 37 and 20 streams leave a workgroup's rows unused;
    37 and 20 span several 16-stream DMA-path workgroups; hysteresis 256 is zc_v2's own)."""
    rng = np.random.default_rng(hyst + n)
    mag = np.abs(rng_c(rng, B, n)) * 0.2
    for b in range(B):
        for p in rng.integers(W, n - 50, size=6):
            mag[b, p:p + rng.integers(1, 40)] += rng.uniform(0.5, 3.0)
    mag[3, n - 5:] += 5.0                              # gate still open at the end
    mt = torch.from_numpy(mag).cuda()
    st, gate, n_ev, ev_i, ev_v = zc_v2._detect_run(mt, W, 200, 15, 0.3, 2048, hyst, 4096)
    for b in range(B):
        so = O.zc_streaming_detection(mag[b], W, 200, 15, 0.3)
        for k in ("local_sum", "corr_scaled", "thresh_scaled"):
            assert np.array_equal(st[k][b].cpu().numpy(), so[k]), k
        assert np.array_equal(st["above_threshold"][b].cpu().numpy().astype(bool), so["above_threshold"])
        assert np.array_equal(st["metric_valid"][b].cpu().numpy().astype(bool), so["metric_valid"])
        evo, valo, masko = O.detect_zc_peaks(mag[b], so["above_threshold"], so["metric_valid"], 2048, hyst)
        k = int(n_ev[b])
        assert k == len(evo) and k > 0
        assert np.array_equal(ev_i[b, :k].cpu().numpy(), evo)
        assert np.array_equal(ev_v[b, :k].cpu().numpy(), valo)
        assert np.array_equal(gate[b].cpu().numpy().astype(bool), masko)


@pytest.mark.parametrize("hyst", [0, 2, 7])
def test_zc_gate_on_given_state(hyst):
    rng = np.random.default_rng(100 + hyst)
    n = 2500
    mag = rng.uniform(0, 1, n)
    above = rng.uniform(0, 1, n) < 0.15
    valid = rng.uniform(0, 1, n) < 0.9               # not monotonic: exercises the skip
    st = zc_v2.ZCDetectionState(corr_mag=mag, local_sum=np.zeros(n), corr_scaled=mag, thresh_scaled=mag,
                                above_threshold=above, metric_valid=valid)
    r = zc_v2.detect_zc_peaks(st, reference_length=300, hysteresis=hyst)
    evo, valo, masko = O.detect_zc_peaks(mag, above, valid, 300, hyst)
    ev = np.array([[e.peak_index, e.gate_start, e.gate_end, e.detected_start] for e in r.events]).reshape(-1, 4)
    assert len(r.events) > 16                         # exercises the event-buffer regrowth
    assert np.array_equal(ev, evo)
    assert np.array_equal([e.peak_value for e in r.events], valo)
    assert np.array_equal(r.gate_mask, masko)


def test_zc_batched_preamble_vs_oracle():
    rng = np.random.default_rng(77)
    B, nb, T = 5, 2, 7000
    ref = O.pss_symbol(2048)
    x = rng_c(rng, B, nb, T) * 0.3
    for b in range(B):
        if b != 2:
            x[b, :, 1000 + 500 * b:1000 + 500 * b + 2048] += ref
    r = zc_v2.detect_zc_preamble_batched(torch.from_numpy(x).cuda(), ref)
    for b in range(B):
        mag = np.abs(sum(O.normalize_correlation(O.matched_filter(x[b, k], ref), x[b, k], ref)
                         for k in range(nb)))
        np.testing.assert_allclose(r.corr_mag[b].cpu().numpy(), mag, rtol=1e-9, atol=1e-12)
        so = O.zc_streaming_detection(r.corr_mag[b].cpu().numpy(), zc_v2.CORR_WINDOW_SIZE, zc_v2.THRESH_VALUE,
                                      zc_v2.THRESH_FRAC_BITS, zc_v2.MIN_CORR_MAG)
        evo, valo, _ = O.detect_zc_peaks(so["corr_mag"], so["above_threshold"], so["metric_valid"], 2048,
                                         zc_v2.HYSTERESIS)
        k = int(r.n_events[b])
        assert np.array_equal(r.events[b, :k].cpu().numpy(), evo)
        if b != 2:      # the preamble's full-overlap peak is among the detections
            assert k >= 1 and np.min(np.abs(evo[:, 0] - (1000 + 500 * b + 2047))) <= 2


def test_zc_combined_batched_vs_oracle():
    rng = np.random.default_rng(3)
    ref = O.pss_symbol(1024)
    x = rng_c(rng, 3, 2, 3000)
    corr, mag = zc.combined_matched_filter_batched(torch.from_numpy(x).cuda(), ref)
    for b in range(3):
        co = O.zc_combined(x[b], ref)
        assert rel(corr[b].cpu().numpy(), co) < 1e-11
        np.testing.assert_allclose(mag[b].cpu().numpy(), np.abs(co), rtol=1e-11, atol=1e-14)


@pytest.mark.parametrize("N,cp,T,nb", [(4096, 0, 4096, 1), (4096, 512, 4620, 2), (2048, 0, 2048, 1),
                                       (1024, 256, 1300, 1), (256, 64, 330, 3), (128, 0, 190, 1)])
def test_zc_freq_fp32_window_fft_vs_oracle(N, cp, T, nb):
    """cfg5 shape (few windows per sequence, complex64): the fp32 window-FFT kernel, every window
    within error model 2 (oracle_zc_freq_check)."""
    from ofdm_sync_amd import _lib
    assert _lib.lib().ofs_zc_freq_plan(_lib.C64, _lib.FP32, T, N, cp) == (3 if N == 4096 else 2)
    rng = np.random.default_rng(N + nb)
    B = 40
    x = rng_c(rng, B, nb, T)
    sym = O.pss_symbol(N)
    for b in range(0, B, 3):                       # every third stream carries the PSS symbol
        x[b, :, cp + (b % 5):cp + (b % 5) + N] += rng.uniform(0.5, 8.0) * sym[:min(N, T - cp - b % 5)]
    x = x.astype(np.complex64)
    idx, t, e = O.zc_template()
    m = zc_freq.compute_frequency_metric_batched(torch.from_numpy(x).cuda(), idx, t, e, N=N, cp=cp)
    assert m.dtype == torch.float32
    mm = m.cpu().numpy()
    st = oracle_c.zc_freq_check(x, N, cp, idx, t, e, mm, EM.zc_win_eps(N), 6.0)
    print(f"zc_freq fp32 N={N} cp={cp} nb={nb}: max |dm| {st[:, 0].max():.3g}, max |dm|/bound {st[:, 1].max():.3g}")
    assert st[:, 1].max() <= 1.0
    mo = O.zc_freq_metric(x[0].astype(np.complex128), N, cp, idx, t, e)      # the numpy oracle agrees
    np.testing.assert_allclose(mm[0], mo, rtol=0, atol=float(st[0, 0]) * 1.01 + 1e-12)
    assert mm.max() > 0.5                          # the PSS windows light up


@pytest.mark.parametrize("B,nb,cp,T", [(1500, 1, 0, 4096), (300, 2, 1, 4099), (70, 3, 6, 4110)])
def test_zc_freq_fp32_lane_reduce_kernel(B, nb, cp, T, variant):
    """N = 4096 lane-reduce kernel (plan 3): persistent grid (B*noff > resident waves), multiple
    branches, odd window starts (direct-load fallback next to the LDS-DMA prefetch).  Against the
    oracle (every stream, error model 2) with both kernels."""
    from ofdm_sync_amd import _lib
    N = 4096
    rng = np.random.default_rng(B + nb)
    x = rng_c(rng, B, nb, T)
    sym = O.pss_symbol(N)
    for b in range(0, B, 4):
        o = b % (T - N - cp + 1)
        x[b, :, cp + o:cp + o + N] += rng.uniform(0.5, 8.0) * sym
    x = x.astype(np.complex64)
    idx, t, e = O.zc_template()
    xd = torch.from_numpy(x).cuda()
    assert _lib.lib().ofs_zc_freq_plan(_lib.C64, _lib.FP32, T, N, cp) == 3
    m = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp).cpu().numpy()
    variant("ZW64", 0)
    assert _lib.lib().ofs_zc_freq_plan(_lib.C64, _lib.FP32, T, N, cp) == 2
    m2 = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp).cpu().numpy()
    for mm, name in ((m, "lane-reduce"), (m2, "transpose")):
        st = oracle_c.zc_freq_check(x, N, cp, idx, t, e, mm, EM.zc_win_eps(N), 6.0)
        print(f"{name} B={B} nb={nb}: max |dm| {st[:, 0].max():.3g}, max |dm|/bound {st[:, 1].max():.3g}")
        assert st[:, 1].max() <= 1.0
    assert m.max() > 0.5


def test_zc_freq_fp32_many_offsets_and_unsupported_shape():
    """complex64 input always returns float32: > 64 offsets per stream run the fp64 sliding DFT
    with the metric rounded to fp32 (plan 5), within u·m of the fp64 kernel's result; shapes the
    block-initialised kernel does not take (3 branches over many offsets) run the one-chunk-per-wave
    fp64 kernel, still with a float32 result (no silent dtype switch, no ValueError)."""
    from ofdm_sync_amd import _lib
    rng = np.random.default_rng(71)
    x = rng_c(rng, 3, 2, 5000).astype(np.complex64)
    x[1, :, 900:900 + 2048] += 3 * O.pss_symbol(2048)
    idx, t, e = O.zc_template()
    assert _lib.lib().ofs_zc_freq_plan(_lib.C64, _lib.FP32, 5000, 2048, 0) == 5
    xd = torch.from_numpy(x).cuda()
    m = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=2048, cp=0)     # auto -> fp32
    assert m.dtype == torch.float32
    m64 = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=2048, cp=0, precision="fp64")
    assert m64.dtype == torch.float64
    mm, m6 = m.cpu().numpy().astype(np.float64), m64.cpu().numpy()
    assert np.all(np.abs(mm - m6) <= 2.0 ** -24 * m6 + 1e-30)          # one rounding to fp32
    st = oracle_c.zc_freq_check(x, 2048, 0, idx, t, e, m.cpu().numpy(), 1e-12, 1.5)
    print(f"fp32 many offsets: max |dm| {st[:, 0].max():.3g}, max |dm|/bound {st[:, 1].max():.3g}")
    assert st[:, 1].max() <= 1.0 and mm[1].max() > 0.5
    # 3 branches x many offsets: not a shape of the block-initialised kernel; the one-chunk-per-wave
    # fp64 kernel takes it with the metric rounded to fp32 (plan 6 for one branch is the same path)
    x3 = rng_c(rng, 2, 3, 3000).astype(np.complex64)
    x3[0, :, 500:500 + 2048] += 3 * O.pss_symbol(2048)
    m3 = zc_freq.compute_frequency_metric_batched(torch.from_numpy(x3).cuda(), idx, t, e, N=2048, cp=0,
                                                  precision="fp32")
    assert m3.dtype == torch.float32
    for b in range(2):
        mo = O.zc_freq_metric(x3[b].astype(np.complex128), 2048, 0, idx, t, e)
        np.testing.assert_allclose(m3[b].cpu().numpy().astype(np.float64), mo, rtol=2.0 ** -22, atol=1e-12)
    assert _lib.lib().ofs_zc_freq_plan(_lib.C64, _lib.FP32, 5000, 2000, 0) == 6        # N % 64 != 0


@pytest.mark.parametrize("fmt,N,cp,T,nb", [("c128", 2048, 512, 16384, 1), ("c128", 2048, 512, 4242, 2),
                                           ("c64", 256, 64, 3001, 1), ("i16", 512, 0, 2600, 2),
                                           ("c128", 64, 16, 700, 1), ("c128", 4096, 1024, 9000, 1),
                                           ("c128", 8192, 0, 8300, 1), ("c128", 192, 5, 1000, 2),
                                           ("c128", 2048, 512, 2600, 1), ("c128", 2048, 512, 8000, 2)])
def test_zc_slide_kernel_vs_oracle_and_previous(fmt, N, cp, T, nb, variant):
    """The block-initialised sliding DFT (zc_slide.hip, plan 4: the pair resonators for the ZC template's
    ±k bins) against the C oracle's fp64 FFTs on every window (1e-9 relative + 1e-11), against the
    per-bin recursion (variant ZS_PAIR=0) and the earlier one-chunk-per-wave kernel (variant ZS=0):
    odd T, cp offsets, chunks past the end, N not a power of two (192), N = 8192 (256-sample
    blocks), offsets fewer than one chunk (T = 2600), int16 and complex64 input, two branches."""
    from ofdm_sync_amd import _lib
    rng = np.random.default_rng(N + T + nb)
    B = 3
    x = rng_c(rng, B, nb, T)
    if T >= 400 + N:
        x[0, :, 300:300 + N] += 3 * O.pss_symbol(N)
    if fmt == "i16":
        xi = np.stack([np.round(x.real * 300), np.round(x.imag * 300)], -1).astype(np.int16)
        xd = torch.from_numpy(xi).cuda()
        x = xi[..., 0] + 1j * xi[..., 1]
    else:
        x = x.astype(np.complex64 if fmt == "c64" else np.complex128)
        xd = torch.from_numpy(x).cuda()
    idx, t, e = O.zc_template()
    assert _lib.lib().ofs_zc_freq_plan({"c128": _lib.C128, "c64": _lib.C64, "i16": _lib.CI16}[fmt], _lib.FP64, T, N,
                                       cp) == 4
    m = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp, precision="fp64").cpu().numpy()
    variant("ZS", 0)
    m_prev = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp, precision="fp64").cpu().numpy()
    variant("ZS", None)
    np.testing.assert_allclose(m, m_prev, rtol=1e-9, atol=1e-11)
    variant("ZS_DEFER", 0)        # per-step DPP row sums instead of the LDS partials
    m_dpp = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp, precision="fp64").cpu().numpy()
    variant("ZS_DEFER", 1)        # LDS partials forced (two branches: only where they fit the block region)
    m_lds = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp, precision="fp64").cpu().numpy()
    variant("ZS_DEFER", None)
    np.testing.assert_allclose(m, m_dpp, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(m, m_lds, rtol=1e-12, atol=1e-14)
    variant("ZS_PAIR", 0)         # first-order recursion per bin instead of the pair resonators
    m_bin = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp, precision="fp64").cpu().numpy()
    variant("ZS_PAIR", None)
    np.testing.assert_allclose(m, m_bin, rtol=1e-9, atol=1e-11)
    for b in range(B):
        mo = O.zc_freq_metric(np.asarray(x[b], np.complex128), N, cp, idx, t, e)
        np.testing.assert_allclose(m[b], mo, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("tmpl,nb", [("zc_shuffled", 1), ("random_pairs", 1), ("random_pairs", 2),
                                     ("unpaired", 1), ("with_dc", 2), ("one_pair", 1)])
def test_zc_slide_templates_pair_and_fallback(tmpl, nb, variant):
    """Template shapes around the pair kernel's condition (every bin k has its mirror N - k, neither
    0 nor N/2): ZC bins in shuffled slot order, random complex template values on paired bins (the
    A/B constants), an unpaired set and a set with the DC bin (both take the per-bin recursion), a
    single pair.  Each against the C oracle's direct DFT (1e-9 relative + 1e-11) and the per-bin
    kernel (variant ZS_PAIR=0)."""
    from ofdm_sync_amd import _lib
    N, cp, T = 2048, 512, 6000
    rng = np.random.default_rng(hash(tmpl) % 1000 + nb)
    idx, t, e = O.zc_template()
    if tmpl == "zc_shuffled":
        perm = rng.permutation(idx.size)
        idx, t = idx[perm], t[perm]
    elif tmpl == "random_pairs":
        k = rng.choice(np.arange(1, 200), 20, replace=False)
        idx = np.concatenate((k, -k))[rng.permutation(40)]
        t = rng_c(rng, idx.size)
    elif tmpl == "unpaired":
        idx = np.arange(1, 40)
        t = rng_c(rng, idx.size)
    elif tmpl == "with_dc":
        idx = np.arange(-20, 21)
        t = rng_c(rng, idx.size)
    elif tmpl == "one_pair":
        idx, t = np.array([-7, 7]), np.array([1.0 + 0.5j, -0.25 + 1j])
    e = float(np.sum(np.abs(t) ** 2))
    x = rng_c(rng, 2, nb, T)
    x[0, :, 700:700 + N] += 3 * O.pss_symbol(N)
    xd = torch.from_numpy(x).cuda()
    m = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp, precision="fp64").cpu().numpy()
    variant("ZS_PAIR", 0)
    m_bin = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp, precision="fp64").cpu().numpy()
    variant("ZS_PAIR", None)
    np.testing.assert_allclose(m, m_bin, rtol=1e-9, atol=1e-11)
    for b in range(2):
        np.testing.assert_allclose(m[b], O.zc_freq_metric(x[b], N, cp, idx, t, e), rtol=1e-9, atol=1e-11)
    assert _lib.lib().ofs_zc_freq_plan(_lib.C128, _lib.FP64, T, N, cp) == 4


@pytest.mark.parametrize("fmt,nb,N,T", [("c128", 1, 2048, 16384), ("c128", 2, 2048, 7000), ("c64", 3, 1024, 3000),
                                        ("int16", 2, 512, 2500), ("c128", 1, 2048, 1000), ("c128", 2, 256, 40),
                                        ("c64", 1, 2048, 9000), ("int16", 1, 2048, 12000)])
def test_zc_fft_overlap_save_equals_direct(fmt, nb, N, T, variant):
    """FFT overlap-save matched filter (ofs_zc_correlate_fft) against the direct sums on the same
    samples, every combine mode: corr within 1e-11 of the row maximum, |corr| 1e-9 relative; for
    8192-point blocks the persistent fused LDS-FFT kernel (default), the one-block-per-workgroup fused
    kernel (variant MC_PERS=0) and the rocFFT pipeline (variant MC_FUSED=0)."""
    rng = np.random.default_rng(N + T + nb)
    B = 3
    x = rng_c(rng, B, nb, T) * 100
    ref = O.pss_symbol(N)
    if T > N + 100:
        x[0, :, 50:50 + N] += 100 * ref
    if fmt == "int16":
        xd = torch.from_numpy(np.stack([np.round(x.real), np.round(x.imag)], -1).astype(np.int16)).cuda()
    else:
        xd = torch.from_numpy(x.astype(np.complex64 if fmt == "c64" else np.complex128)).cuda()
    for fused in ("1", "1block", "0"):
        variant("MC_FUSED", 0 if fused == "0" else 1)
        variant("MC_PERS", 0 if fused == "1block" else None)
        for mode in (zc_v2.OFS_ZC_RAW, zc_v2.OFS_ZC_V2, zc_v2.OFS_ZC_COMBINED, zc_v2.OFS_ZC_SUM):
            cf, mf = zc_v2.correlate_batched(xd, ref, mode, want_corr=True, want_mag=True, method="fft")
            cd, md = zc_v2.correlate_batched(xd, ref, mode, want_corr=True, want_mag=True, method="direct")
            cf, cd, mf, md = cf.cpu().numpy(), cd.cpu().numpy(), mf.cpu().numpy(), md.cpu().numpy()
            scale = np.abs(cd).max(axis=-1, keepdims=True)
            assert np.max(np.abs(cf - cd) / scale) < 1e-11, (mode, fused)
            np.testing.assert_allclose(mf, md, rtol=1e-9, atol=1e-11 * float(scale.max()))
    variant("MC_FUSED", None)
    variant("MC_PERS", None)


@pytest.mark.parametrize("fmt,nb,B,T", [("c128", 1, 300, 16384), ("c64", 1, 97, 20000), ("c128", 2, 150, 16384),
                                        ("int16", 1, 700, 5000)])
def test_zc_fft_persistent_kernel_many_blocks(fmt, nb, B, T, variant):
    """The persistent matched-filter kernel (zc_fftcorr.hip mc_pers_kernel: one workgroup per CU walking
    a run of 8192-point blocks, the next block's input prefetched during the current one) on batches
    of more blocks than CUs, runs of unequal length and runs that cross stream boundaries: equal to
    the one-block-per-workgroup kernel (variant MC_PERS=0) within 1e-12 of the row maximum, and to
    the direct sums on sampled streams (1e-11 / |corr| 1e-9 relative), every output."""
    rng = np.random.default_rng(B + T + nb)
    ref = O.pss_symbol(2048)
    x = rng_c(rng, B, nb, T) * 100
    for b in range(0, B, 7):
        s0 = int(rng.integers(0, T - 2048))
        x[b, :, s0:s0 + 2048] += 100 * ref
    if fmt == "int16":
        xd = torch.from_numpy(np.stack([np.round(x.real), np.round(x.imag)], -1).astype(np.int16)).cuda()
    else:
        xd = torch.from_numpy(x.astype(np.complex64 if fmt == "c64" else np.complex128)).cuda()
    for mode in (zc_v2.OFS_ZC_V2, zc_v2.OFS_ZC_RAW):
        cp, mp = zc_v2.correlate_batched(xd, ref, mode, want_corr=True, want_mag=True, method="fft")
        variant("MC_PERS", 0)
        c1, m1 = zc_v2.correlate_batched(xd, ref, mode, want_corr=True, want_mag=True, method="fft")
        variant("MC_PERS", None)
        scale = c1.abs().amax(dim=-1, keepdim=True)
        assert float(((cp - c1).abs() / scale).max()) < 1e-12, mode
        np.testing.assert_allclose(mp.cpu().numpy(), m1.cpu().numpy(), rtol=1e-9, atol=1e-12 * float(scale.max()))
        rows = torch.arange(0, B, max(1, B // 6), device=xd.device)
        cd, md = zc_v2.correlate_batched(xd[rows], ref, mode, want_corr=True, want_mag=True, method="direct")
        sc = cd.abs().amax(dim=-1, keepdim=True)
        assert float(((cp[rows] - cd).abs() / sc).max()) < 1e-11, mode
        np.testing.assert_allclose(mp[rows].cpu().numpy(), md.cpu().numpy(), rtol=1e-9,
                                   atol=1e-11 * float(sc.max()))


def test_zc_detect_four_branches_n2048_falls_back_to_direct():
    """4 branches x 2048 taps: the overlap-save extract cannot hold the branches' energy prefixes
    in LDS (ofs_zc_mf_plan_create -> OFS_ETOOLONG); method="auto" takes the direct sums (the
    reference's detect_zc_preamble takes any branch count, zc_v2.py:452-519), method="fft" raises."""
    rng = np.random.default_rng(44)
    B, nb, T = 2, 4, 6000
    ref = O.pss_symbol(2048)
    x = rng_c(rng, B, nb, T) * 0.3
    x[0, :, 1500:1500 + 2048] += ref
    xd = torch.from_numpy(x).cuda()
    with pytest.raises(RuntimeError):
        zc_v2.correlate_batched(xd, ref, zc_v2.OFS_ZC_V2, want_corr=False, want_mag=True, method="fft")
    r = zc_v2.detect_zc_preamble_batched(xd, ref)
    for b in range(B):
        mag = np.abs(sum(O.normalize_correlation(O.matched_filter(x[b, k], ref), x[b, k], ref) for k in range(nb)))
        np.testing.assert_allclose(r.corr_mag[b].cpu().numpy(), mag, rtol=1e-9, atol=1e-12)
    k = int(r.n_events[0])
    assert k >= 1 and np.min(np.abs(r.events[0, :k, 0].cpu().numpy() - (1500 + 2047))) <= 2


def test_zc_fft_plan_cache_device_references_at_recycled_address():
    """Two different same-length device references allocated back to back, the first freed before
    the second exists, so torch's caching allocator gives the second the first's address (and the
    same version counter 0): the plan cache keys by content, so each call correlates with its own
    reference and equals the oracle (a key on data_ptr/_version returned the first plan's spectrum)."""
    rng = np.random.default_rng(46)
    x = rng_c(rng, 2, 1, 9000)
    xd = torch.from_numpy(x).cuda()
    ptrs = []
    for root in (25, 29, 34):
        ref_h = O.pss_symbol(2048, root=root)
        x_r = x.copy()
        x_r[0, 0, 3000:3000 + ref_h.size] += ref_h
        xd.copy_(torch.from_numpy(x_r))
        ref_d = torch.as_tensor(ref_h, device="cuda")
        ptrs.append(ref_d.data_ptr())
        _, mag = zc_v2.correlate_batched(xd, ref_d, zc_v2.OFS_ZC_V2, want_corr=False, want_mag=True, method="fft")
        mag = mag.cpu().numpy()
        del ref_d
        for b in range(2):
            want = np.abs(O.normalize_correlation(O.matched_filter(x_r[b, 0], ref_h), x_r[b, 0], ref_h))
            np.testing.assert_allclose(mag[b], want, rtol=1e-9, atol=1e-12)
    assert len(set(ptrs)) < len(ptrs), "the allocator did not recycle the address; the test is vacuous"


@pytest.mark.parametrize("method", ["fft", "direct"])
def test_zc_matched_filter_handle_skips_host_copy(method, monkeypatch):
    """zc_v2.MatchedFilter: the prepared reference gives the same correlation and detection as the
    raw taps (bit for bit), and a call with it never copies / hashes the taps again (the per-call
    device-to-host sync of a raw device reference): _ref_host is made to fail after construction."""
    rng = np.random.default_rng(47)
    ref_h = O.pss_symbol(2048, root=29)
    x = rng_c(rng, 3, 1, 9000)
    x[1, 0, 4000:4000 + ref_h.size] += 2 * ref_h
    xd = torch.from_numpy(x).cuda()
    mf = zc_v2.MatchedFilter(torch.as_tensor(ref_h, device="cuda"))
    assert len(mf) == ref_h.size
    want_c, want_m = zc_v2.correlate_batched(xd, ref_h, zc_v2.OFS_ZC_V2, want_mag=True, method=method)
    want_d = zc_v2.detect_zc_preamble_batched(xd, ref_h)

    def _no_copy(*a, **k):
        raise AssertionError("reference copied to the host")
    monkeypatch.setattr(zc_v2, "_ref_host", _no_copy)
    got_c, got_m = zc_v2.correlate_batched(xd, mf, zc_v2.OFS_ZC_V2, want_mag=True, method=method)
    assert torch.equal(got_c, want_c) and torch.equal(got_m, want_m)
    got_d = zc_v2.detect_zc_preamble_batched(xd, mf)
    assert torch.equal(got_d.n_events, want_d.n_events) and int(got_d.n_events[1]) >= 1
    k = int(want_d.n_events[1])
    assert torch.equal(got_d.events[1, :k], want_d.events[1, :k])
    assert torch.equal(mf.correlate(xd, want_mag=True, method=method)[1], want_m)


def test_zc_fft_plan_shared_by_two_streams():
    """One cached overlap-save plan used from two HIP streams back to back: each call takes its own
    scratch / work buffers from torch's stream-ordered allocator, so the results equal the
    single-stream results bit for bit."""
    rng = np.random.default_rng(45)
    ref = O.pss_symbol(2048)
    xs = [torch.from_numpy(rng_c(rng, 4, 1, 9000)).cuda() for _ in range(2)]
    want = [zc_v2.correlate_batched(x, ref, zc_v2.OFS_ZC_V2, want_mag=True, method="fft")[1].clone() for x in xs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for _ in range(3):
        for x, s in zip(xs, streams):
            with torch.cuda.stream(s):
                got.append(zc_v2.correlate_batched(x, ref, zc_v2.OFS_ZC_V2, want_mag=True, method="fft")[1])
    torch.cuda.synchronize()
    for i, g in enumerate(got):
        assert torch.equal(g, want[i % 2])


@pytest.mark.parametrize("fmt,nb,nbins,N,cp,T", [("c128", 6, 62, 256, 64, 1500), ("c128", 1, 100, 256, 32, 900),
                                                 ("c64", 6, 100, 128, 16, 700), ("c64", 3, 62, 256, 64, 1500),
                                                 ("c64", 4, 62, 200, 20, 900), ("int16", 5, 70, 192, 0, 800),
                                                 ("c128", 9, 130, 64, 16, 300)])
def test_zc_freq_any_branches_and_bins(fmt, nb, nbins, N, cp, T):
    """zc_freq.py:62-99 loops over any number of branches and template bins: more than 4 branches
    or 64 bins run as partial sums over groups of <= 4 x <= 64 (ofs_zc_freq_partial + _finish);
    complex64 with 3-4 branches or N not a multiple of 64 over many offsets falls back to the
    one-chunk-per-wave fp64 kernel with an fp32 metric.  Against the oracle: 1e-9 relative for fp64
    output, fp32 rounding of the fp64 metric (2^-23 relative) for complex64."""
    rng = np.random.default_rng(nb * 100 + nbins)
    B = 3
    x = rng_c(rng, B, nb, T)
    x[1, :, 100:100 + N] += 3 * O.pss_symbol(N, length=min(62, N - 2 - (N % 2)))
    half = nbins // 2
    idx = np.concatenate((np.arange(-half, 0), np.arange(1, nbins - half + 1)))
    t = np.exp(-1j * np.pi * 25 * np.arange(nbins) * (np.arange(nbins) + 1) / nbins)
    e = float(np.sum(np.abs(t) ** 2))
    if fmt == "int16":
        xi = np.stack([np.round(x.real * 100), np.round(x.imag * 100)], -1).astype(np.int16)
        xd, x = torch.from_numpy(xi).cuda(), xi[..., 0] + 1j * xi[..., 1]
    elif fmt == "c64":
        x = x.astype(np.complex64)
        xd = torch.from_numpy(x).cuda()
    else:
        xd = torch.from_numpy(x).cuda()
    m = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp)
    assert m.dtype == (torch.float32 if fmt == "c64" else torch.float64)
    m = m.cpu().numpy().astype(np.float64)
    for b in range(B):
        mo = O.zc_freq_metric(x[b].astype(np.complex128), N, cp, idx, t, e)
        if fmt == "c64":
            np.testing.assert_allclose(m[b], mo, rtol=2.0 ** -22, atol=1e-12)
        else:
            np.testing.assert_allclose(m[b], mo, rtol=1e-9, atol=1e-11)
    if fmt != "c64":                       # the drop-in: numpy in, reference globals for N / cp
        import ofdm_sync_amd.zc_freq as zf
        old = (zf.N_FFT, zf.CYCLIC_PREFIX)
        zf.N_FFT, zf.CYCLIC_PREFIX = N, cp
        try:
            m1 = zf.compute_frequency_metric(x[1], idx, t, e)
        finally:
            zf.N_FFT, zf.CYCLIC_PREFIX = old
        np.testing.assert_allclose(m1, O.zc_freq_metric(x[1].astype(np.complex128), N, cp, idx, t, e),
                                   rtol=1e-9, atol=1e-11)
