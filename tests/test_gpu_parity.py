"""GPU parity: every drop-in entry point (through the C ABI of libofdmsync.so) against the
reference's golden vectors and the CPU oracle.

Tolerances (written here, per north_star):
  fp64 path (complex128 / int16 input): P, R within 1e-11 relative to the stream maximum,
      M within 1e-12 absolute, event indices exact; integer (int12) inputs bit-exact where the
      reference is integer-exact (aa P, every minn_rtl array).
  fp32 path (complex64 input): M within 1e-6 absolute (north_star), P and R within 1e-5
      relative to the stream maximum; events exact except stated near-ties (oracle/parity.py:
      above flags may differ only where |M - thr| <= 1e-6, gate bounds exact under the
      engine's flags, peak within 1e-5 relative |P|^2 of the gate max, CFO angle <= 1e-6 rad).
"""
import glob
import os

import numpy as np
import pytest

import ofdm_oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - the -m gpu run is on the GPU box
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import sync_aa, sc, minn, minn_rtl, combined_sc_min, core, _lib  # noqa: E402
from test_oracle_golden import _csv_rows, _fmt_rows, unsign_zero  # noqa: E402
from aa_check import check_fp32_batch  # noqa: E402


def G(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def cases(kind):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        if str(np.load(p)["kind"]) == kind:
            out.append(os.path.basename(p)[:-4])
    return out


def relerr(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def test_native_library_is_the_one_loaded():
    L = _lib.lib()
    assert os.path.samefile(L._name, _lib.LIB_PATH)
    maps = open("/proc/self/maps").read()
    assert "libofdmsync.so" in maps


# ------------------------------------------------------------------ sync_aa ------------
@pytest.mark.parametrize("name", cases("aa"))
def test_aa_fp64_vs_reference_golden(name):
    d = G(name)
    r = sync_aa.aa_detect_streaming(d["x"], L=int(d["L"]), threshold=float(d["threshold"]),
                                    hysteresis=int(d["hysteresis"]), sample_rate=float(d["sample_rate"]))
    st = r.state
    assert st.P.dtype == np.complex128 and st.M.dtype == np.float64
    assert relerr(st.P, d["P"]) < 1e-11
    assert relerr(st.R, d["R"]) < 1e-11
    assert np.max(np.abs(st.M - d["M"]), initial=0) < 1e-12
    assert np.array_equal(st.valid, d["valid"])
    assert r.num_antennas == d["x"].shape[0]
    ei = np.array([[e.peak_index, e.gate_start, e.gate_end, e.frame_start] for e in r.events]).reshape(-1, 4)
    er = np.array([[e.P_at_peak.real, e.P_at_peak.imag, e.M_at_peak, e.cfo_hz] for e in r.events]).reshape(-1, 4)
    assert np.array_equal(ei, d["ev_int"])
    assert np.allclose(er, d["ev_real"], rtol=1e-10, atol=1e-8)
    if "int12" in name:
        assert np.array_equal(st.P, d["P"])      # exact integer sums


@pytest.mark.parametrize("csv,case", [("detector_test_vector.csv", "aa_clean_L512"),
                                      ("detector_cfo_test_vector.csv", "aa_cfo_L512")])
def test_aa_reproduces_reference_csv_on_gpu(csv, case):
    header, rows = _csv_rows(csv)
    d = G(case)
    r = sync_aa.aa_detect_streaming(d["x"], L=512)
    idx = [int(row.split(",")[0]) for row in rows]
    got = _fmt_rows(r.state.P, r.state.R, r.state.M, header.split(","), idx)
    assert [unsign_zero(g) for g in got] == [unsign_zero(w) for w in rows]
    assert r.events[0].peak_index == 1523 and r.events[0].frame_start == 500
    if "cfo" in csv:
        assert abs(r.events[0].cfo_hz - 500.0) < 1e-6


@pytest.mark.parametrize("name", ["aa_clean_L512", "aa_cfo_L512", "aa_grid_len1024_awgn_snr10_fs1.0",
                                  "aa_grid_len512_cir2_snr5_fs2.0", "aa_grid_len1024_cir1_snr0_fs0.5",
                                  "aa_grid_len256_cir1_snr0_fs1.0"])
def test_aa_fp32_vs_reference_golden(name):
    """fp32 engine on the reference's own detector inputs (sync_aa.run_single_test: ~2-5.3k
    samples, 2 antennas): wave-per-stream plan (register-staged or streaming), metric within
    1e-6, every event exact under oracle/parity.py's near-tie criterion against the
    REFERENCE's outputs."""
    d = G(name)
    x = d["x"].astype(np.complex64)
    na, T = x.shape
    L = int(d["L"])
    assert _lib.lib().ofs_aa_plan(_lib.C64, _lib.FP32, na, T, L) >= 1000
    out = sync_aa.aa_detect_streaming_batched(torch.from_numpy(x[None]).cuda(), L=L, threshold=float(d["threshold"]),
                                              hysteresis=int(d["hysteresis"]), sample_rate=float(d["sample_rate"]))
    assert out.M.dtype == torch.float32
    ref = [(d["P"], d["R"], d["M"], d["valid"], d["ev_int"].reshape(-1, 4), d["ev_real"].reshape(-1, 4))]
    r = check_fp32_batch(out, x[None], L, float(d["threshold"]), int(d["hysteresis"]), float(d["sample_rate"]), ref)
    assert r["exact"] == 1
    # the reference-precision (complex128) path of the same input: wave-per-stream at any T
    assert _lib.lib().ofs_aa_plan(_lib.C128, _lib.FP64, na, T, L) >= 3000


def test_aa_int16_iq_input_exact():
    d = G("aa_int12_L128")
    x = d["x"]
    iq = np.stack([x.real, x.imag], axis=-1).astype(np.int16)[None]        # [1, 2, T, 2]
    out = sync_aa.aa_detect_streaming_batched(torch.from_numpy(iq).cuda(), L=128)
    assert out.P.dtype == torch.complex128
    assert np.array_equal(out.P[0].cpu().numpy(), d["P"])
    Pq, Rq, Mq, _ = O.aa_metric(x, 128)
    assert np.array_equal(out.R[0].cpu().numpy(), Rq)                         # re²+im² integers
    assert np.max(np.abs(out.M[0].cpu().numpy() - d["M"])) < 1e-12
    assert int(out.n_events[0]) == len(d["ev_int"])
    assert np.array_equal(out.ev_int[0, :len(d["ev_int"])].cpu().numpy(), d["ev_int"])


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
@pytest.mark.parametrize("seed", range(6))
def test_aa_batched_random_vs_oracle(seed, prec):
    rng = np.random.default_rng(100 + seed)
    B = int(rng.integers(1, 40))
    nb = int(rng.integers(1, 4))
    T = int(rng.choice([1, 7, 64, 513, 1024, 2048, 3000, 4500, 9000]))
    L = int(rng.choice([1, 3, 32, 128, 256, 512, 1000]))
    x = rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))
    # plant an [A][A] burst in half the streams so gates open
    for b in range(0, B, 2):
        if T >= 2 * L + 10:
            s = int(rng.integers(0, T - 2 * L))
            a = (rng.standard_normal(L) + 1j * rng.standard_normal(L)) * 3
            x[b, :, s:s + L] += a
            x[b, :, s + L:s + 2 * L] += a
    xt = torch.from_numpy(x if prec == "fp64" else x.astype(np.complex64)).cuda()
    thr, hyst = 0.2, int(rng.choice([1, 5, 64]))
    out = sync_aa.aa_detect_streaming_batched(xt, L=L, threshold=thr, hysteresis=hyst, precision=prec)
    P, R, M = out.P.cpu().numpy(), out.R.cpu().numpy(), out.M.cpu().numpy()
    nev = out.n_events.cpu().numpy()
    for b in range(B):
        xb = x[b] if prec == "fp64" else x[b].astype(np.complex64).astype(np.complex128)
        Pr, Rr, Mr, vr, ei, er = O.aa_detect(xb, L, thr, hyst)
        if prec == "fp64":
            assert relerr(P[b], Pr) < 1e-11 and relerr(R[b], Rr) < 1e-11
            assert np.max(np.abs(M[b] - Mr), initial=0) < 1e-12
            assert nev[b] == len(ei)
            assert np.array_equal(out.ev_int[b, :nev[b]].cpu().numpy(), ei)
            assert np.allclose(out.ev_real[b, :nev[b]].cpu().numpy(), er, rtol=1e-9, atol=1e-7)
        assert np.array_equal(out.valid[b].cpu().numpy(), vr)
    if prec == "fp32":
        check_fp32_batch(out, x.astype(np.complex64), L, thr, hyst)


def test_aa_edge_lengths():
    r = sync_aa.aa_detect_streaming(np.zeros(0, complex), L=8)
    assert r.events == [] and r.state.M.size == 0
    r = sync_aa.aa_detect_streaming(np.ones(5, complex), L=8)
    assert not r.state.valid.any() and np.all(r.state.M == 0) and r.events == []
    # constant input: M == 1 everywhere valid, one unclosed gate, first max wins
    r = sync_aa.aa_detect_streaming(np.ones(64, complex), L=8, threshold=0.5, hysteresis=3)
    Pr, Rr, Mr, vr, ei, er = O.aa_detect(np.ones(64, complex), 8, 0.5, 3)
    assert np.array_equal([[e.peak_index, e.gate_start, e.gate_end, e.frame_start] for e in r.events], ei)


def test_aa_many_events_grow_buffer():
    """More events than the initial event buffer: the wrapper re-runs with room for all."""
    T, L = 6000, 4
    x = np.zeros(T, complex)
    for k in range(40):
        s = 100 + 140 * k
        x[s:s + 2 * L] = 1.0
    r = sync_aa.aa_detect_streaming(x, L=L, threshold=0.5, hysteresis=3)
    Pr, Rr, Mr, vr, ei, er = O.aa_detect(x, L, 0.5, 3)
    assert len(r.events) == len(ei) > 16
    assert np.array_equal([[e.peak_index, e.gate_start, e.gate_end, e.frame_start] for e in r.events], ei)


# ------------------------------------------------------- sc / combined / minn ------------
def _window_call(kind, x, N, prec=None):
    if kind == "sc":
        old = sc.N_FFT
        sc.N_FFT = N
        try:
            return sc.sc_streaming_metric(x, precision=prec)
        finally:
            sc.N_FFT = old
    if kind == "comb_sc":
        return combined_sc_min.schmidl_cox_streaming_metric(x, symbol_len=N, precision=prec)
    return minn.minn_streaming_metric_parameterized(x, N, precision=prec)


@pytest.mark.parametrize("name", cases("sc") + cases("comb_sc") + cases("minn"))
def test_window_metrics_fp64_vs_reference_golden(name):
    d = G(name)
    kind = str(d["kind"])
    M, P, R = _window_call(kind, d["x"], int(d["N"]))
    assert M.shape == d["M"].shape and P.dtype == np.complex128
    if M.size:
        assert relerr(P, d["P"]) < 1e-11
        assert relerr(R, d["R"]) < 1e-11
        assert np.max(np.abs(M - d["M"])) < 1e-10


@pytest.mark.parametrize("name", ["sc_N64_cfg1", "sc_N2048_cir1", "sc_N1024_cir2_2br",
                                  "comb_sc_N2048_cir1_2br", "comb_minn_N2048_cir1_2br", "minn_param_N256"])
def test_window_metrics_fp32_vs_reference_golden(name):
    d = G(name)
    kind = str(d["kind"])
    x = torch.from_numpy(d["x"].astype(np.complex64)).cuda()
    M, P, R = _window_call(kind, x, int(d["N"]))
    assert M.dtype == torch.float32
    assert np.max(np.abs(M.cpu().numpy() - d["M"])) < 1e-6
    assert relerr(P.cpu().numpy(), d["P"]) < 1e-5
    assert relerr(R.cpu().numpy(), d["R"]) < 1e-5


def test_module_global_n_fft_is_read_at_call_time():
    d = G("sc_N64_cfg1")
    sc.N_FFT = 64
    try:
        M, P, R = sc.sc_streaming_metric(d["x"])
    finally:
        sc.N_FFT = 2048
    assert np.max(np.abs(M - d["M"])) < 1e-10
    d = G("comb_minn_N2048_cir1_2br")
    M, P, R = combined_sc_min.minn_streaming_metric(d["x"])
    assert np.max(np.abs(M - d["M"])) < 1e-10
    M, P, R = minn.minn_streaming_metric(d["x"])
    assert np.max(np.abs(M - d["M"])) < 1e-10


def test_window_metric_edges():
    x = np.ones((2, 100), complex)
    old = sc.N_FFT
    sc.N_FFT = 128
    try:
        M, P, R = sc.sc_streaming_metric(x)
        assert M.size == 0 and P.size == 0 and R.size == 0
        sc.N_FFT = 63
        with pytest.raises(ValueError):
            sc.sc_streaming_metric(x)
    finally:
        sc.N_FFT = old
    M, P, R = combined_sc_min.schmidl_cox_streaming_metric(x, symbol_len=1)
    assert M.size == 0
    M, P, R = minn.minn_streaming_metric_parameterized(x, 3)   # Q = 0: zero metric
    Mr, Pr, Rr = O.minn_metric(x, 3)
    assert np.array_equal(M, Mr) and np.allclose(P, Pr)


@pytest.mark.parametrize("seed", range(4))
def test_window_metrics_batched_random(seed):
    rng = np.random.default_rng(7 + seed)
    B, nb = int(rng.integers(1, 20)), int(rng.integers(1, 3))
    T = int(rng.choice([300, 2048, 5000, 7000]))
    N = int(rng.choice([16, 64, 256, 1024, 2048]))
    x = rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))
    xt = torch.from_numpy(x).cuda()
    for kind, fn in (("sc", sc.sc_streaming_metric_batched),
                     ("comb_sc", combined_sc_min.schmidl_cox_streaming_metric_batched),
                     ("minn", minn.minn_streaming_metric_batched)):
        M, P, R = fn(xt, N)
        ofn = {"sc": O.sc_metric, "comb_sc": O.comb_sc_metric, "minn": O.minn_metric}[kind]
        for b in range(B):
            Mr, Pr, Rr = ofn(x[b], N)
            assert relerr(P[b].cpu().numpy(), Pr) < 1e-11, kind
            assert np.max(np.abs(M[b].cpu().numpy() - Mr), initial=0) < 1e-10, kind


# ---------------------------------------------------------------- minn_rtl ------------
RTL_KEYS = ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled",
            "energy_scaled", "metric_valid", "above_threshold")


@pytest.mark.parametrize("name", cases("minn_rtl"))
def test_minn_rtl_vs_reference_golden(name):
    d = G(name)
    st = minn_rtl.minn_rtl_streaming_metric(
        d["x"], smooth_shift=int(d["smooth_shift"]), threshold_value=int(d["threshold_value"]),
        threshold_frac_bits=int(d["threshold_frac_bits"]), quarter_len=int(d["Q"]))
    exact = "int12" in name
    for k in RTL_KEYS:
        got = getattr(st, k)
        if exact:
            assert np.array_equal(got, d[k]), k          # bit-exact integer path
        else:
            assert np.allclose(got, d[k], rtol=1e-9, atol=1e-6), k
    det = minn_rtl.detect_minn_rtl(st, hysteresis=int(d["hysteresis"]), timing_offset=int(d["timing_offset"]))
    ev = np.array([[e.peak_index, e.detected_index, *e.gate_segment] for e in det.events]).reshape(-1, 4)
    assert np.array_equal(ev, d["events"])
    assert np.array_equal(np.array(det.gate_segments).reshape(-1, 2), d["gate_segments"])
    assert np.array_equal(det.gate_mask, d["gate_mask"])


@pytest.mark.parametrize("name", ["rtl_Q64_int12", "rtl_Q512_int12", "rtl_Q64_int12_noshift_h0"])
def test_minn_rtl_batched_int16_fused_gate(name):
    d = G(name)
    x = d["x"]
    iq = np.stack([x.real, x.imag], axis=-1).astype(np.int16)
    iq = np.stack([iq, iq[:, ::-1].copy()])          # second stream = time-reversed copy
    out = minn_rtl.minn_rtl_batched(torch.from_numpy(iq).cuda(), int(d["Q"]),
                                    smooth_shift=int(d["smooth_shift"]), threshold_value=int(d["threshold_value"]),
                                    threshold_frac_bits=int(d["threshold_frac_bits"]),
                                    hysteresis=int(d["hysteresis"]), timing_offset=int(d["timing_offset"]))
    for k in RTL_KEYS:
        assert np.array_equal(getattr(out, k)[0].cpu().numpy(), d[k]), k
    n = int(out.n_events[0])
    assert np.array_equal(out.events[0, :n].cpu().numpy(), d["events"])
    xr = (iq[1, ..., 0] + 1j * iq[1, ..., 1]).astype(np.complex128)
    s = O.minn_rtl_metric(xr, int(d["Q"]), int(d["smooth_shift"]), int(d["threshold_value"]), int(d["threshold_frac_bits"]))
    for k in RTL_KEYS:
        assert np.array_equal(getattr(out, k)[1].cpu().numpy(), s[k]), k
    ev, seg, mask = O.detect_minn_rtl(s["corr_positive"], s["above_threshold"], s["metric_valid"],
                                      int(d["hysteresis"]), int(d["timing_offset"]))
    n1 = int(out.n_events[1])
    assert np.array_equal(out.events[1, :n1].cpu().numpy(), ev)


def test_minn_rtl_floor_mode_matches_oracle():
    d = G("rtl_Q64_int12")
    st = minn_rtl.minn_rtl_streaming_metric(d["x"], smooth_shift=3, threshold_value=3276,
                                            threshold_frac_bits=15, quarter_len=64, smooth_mode="floor")
    s = O.minn_rtl_metric(d["x"], 64, 3, 3276, 15, smooth_mode="floor")
    for k in RTL_KEYS:
        assert np.array_equal(getattr(st, k), s[k]), k


def test_minn_rtl_rejects_bad_quarter():
    with pytest.raises(ValueError):
        minn_rtl.minn_rtl_streaming_metric(np.ones(10), smooth_shift=3, threshold_value=1,
                                           threshold_frac_bits=15, quarter_len=0)


# ---------------------------------------------------------------- CP CFO ------------
def test_cp_cfo_vs_reference_golden():
    d = G("cp_cfo")
    got = [core.estimate_cfo_from_cp(d["x"], int(s), int(d["n_fft"]), int(d["cp_len"]), float(d["fs"]))
           for s in d["starts"]]
    assert np.allclose(got, d["cfo"], rtol=0, atol=1e-9)
    got1 = [core.estimate_cfo_from_cp(d["x"][0], int(s), 2048, 256, float(d["fs_1br"])) for s in d["starts"]]
    assert np.allclose(got1, d["cfo_1br_cp256"], rtol=0, atol=1e-9)
    xb = torch.from_numpy(np.stack([d["x"]] * len(d["starts"]))).cuda()
    c = core.estimate_cfo_from_cp_batched(xb, d["starts"], 2048, 512, float(d["fs"]))
    assert np.allclose(c.cpu().numpy(), d["cfo"], rtol=0, atol=1e-9)


def test_cp_search_vs_reference_golden():
    """core.py:199-336 searches: CFO within 1e-8 Hz, indices exact, fallbacks as the reference."""
    d = G("cp_search")
    x, N, cp, fs = d["x"], int(d["n_fft"]), int(d["cp_len"]), float(d["fs"])
    est = [int(e) for e in d["est"]]
    close = lambda a, b: np.allclose(a, b, rtol=0, atol=1e-8)   # noqa: E731
    assert close([core.estimate_cfo_from_cp_robust(x, e, N, cp, fs) for e in est], d["robust"])
    assert close([core.estimate_cfo_from_cp_robust(x, e, N, cp, fs, span=40, win_len=100) for e in est],
                 d["robust_s40_w100"])
    assert close([core.estimate_cfo_from_cp_robust(x[0], e, N, cp, fs, span=0) for e in est], d["robust_1br_s0"])
    pk = [core.estimate_cfo_from_cp_peak_with_index(x, e, N, cp, fs) for e in est]
    assert close([p[0] for p in pk], d["peak_cfo"]) and [p[1] for p in pk] == list(d["peak_d"])
    assert close([core.estimate_cfo_from_cp_peak(x, e, N, cp, fs) for e in est], d["peak_only"])
    pk = [core.estimate_cfo_from_cp_peak_with_index(x[1], e, N, 256, fs, span=300) for e in est]
    assert close([p[0] for p in pk], d["peak_1br_s300_cfo"]) and [p[1] for p in pk] == list(d["peak_1br_s300_d"])
    assert [core.find_cp_start_via_corr(x, e, N, cp) for e in est] == list(d["find_start"])
    assert [core.find_cp_start_via_corr(x, e, N, cp, search_half=64) for e in est] == list(d["find_start_h64"])


@pytest.mark.parametrize("fmt", ["c64", "c128", "int16"])
def test_cp_search_batched_vs_oracle(fmt):
    """Batched search over many streams and input formats against the oracle loops."""
    rng = np.random.default_rng(3)
    B, nb, T, N, cp = 24, 2, 1500, 512, 128
    x = (rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))) * 200
    x[:, :, 700:700 + cp] += x[:, :, 700 + N:700 + N + cp]          # a CP-like repeat per stream
    x = np.round(x)
    est = rng.integers(0, T, B)
    est[:3] = (0, T - N - cp, T - 1)
    if fmt == "int16":
        xi = np.stack([x.real, x.imag], -1).astype(np.int16)
        xd = torch.from_numpy(xi).cuda()
    else:
        xd = torch.from_numpy(x.astype(np.complex64 if fmt == "c64" else np.complex128)).cuda()
    xr = x.astype(np.complex64).astype(np.complex128) if fmt == "c64" else x
    for mode, win, span in ((core.CPS_ROBUST, 64, 40), (core.CPS_PEAK, cp, 200)):
        cfo, d, _, st = core.cp_search_batched(xd, est, N, win, span, mode, 1e6)
        cfo, d, st = cfo.cpu().numpy(), d.cpu().numpy(), st.cpu().numpy()
        for b in range(B):
            lo, hi = max(0, est[b] - span), min(T - (N + win), est[b] + span)
            assert st[b] == (1 if hi <= lo else 0)
            if st[b]:
                assert d[b] == est[b]
                continue
            if mode == core.CPS_ROBUST:
                ref = O.cp_cfo_robust(xr[b], int(est[b]), N, 2 * win, 1e6, span=span, win_len=win)
                assert abs(cfo[b] - ref) < 1e-6
            else:
                rc, rd = O.cp_cfo_peak(xr[b], int(est[b]), N, win, 1e6, span=span)
                assert d[b] == rd and abs(cfo[b] - rc) < 1e-6


# ------------------------------------------------------- full-size (BASELINE cfg3) ------------
def test_aa_fp32_full_batch_properties():
    """B = 65536 streams x T = 1024 c64, L = 512: oracle on a sample of streams, invariants
    on all of them (valid mask, 0 <= M <= 1, scale invariance of M, P/R scale as |a|²)."""
    B, T, L = 65536, 1024, 512
    g = torch.Generator(device="cuda").manual_seed(1234)
    x = torch.randn((B, 1, T), dtype=torch.complex64, device="cuda", generator=g)
    x[:, :, 512:] += x[:, :, :512].clone()            # [A][A]-like correlation in every stream
    out = sync_aa.aa_detect_streaming_batched(x, L=L, precision="fp32")
    M = out.M
    assert bool((M[:, :L] == 0).all()) and bool((M >= 0).all()) and bool((M <= 1).all())
    assert bool(out.valid[:, L:].all()) and not bool(out.valid[:, :L].any())
    idx = torch.randint(0, B, (48,), generator=g, device="cuda").cpu().numpy()
    xs = x[idx].cpu().numpy().astype(np.complex128)
    for k, b in enumerate(idx):
        Pr, Rr, Mr, vr = O.aa_metric(xs[k], L)
        assert np.max(np.abs(M[b].cpu().numpy() - Mr)) < 1e-6
    out2 = sync_aa.aa_detect_streaming_batched(x * 2, L=L, precision="fp32")
    assert torch.max(torch.abs(out2.M - M)).item() < 1e-6
    assert torch.allclose(out2.R, 4 * out.R, rtol=1e-5)
    # every stream has its gate open at the end (correlated second half) -> >= 1 event
    assert bool((out.n_events >= 1).all())


# ------------------------------------------------------- fast path (aa_fast_kernel) ------------
@pytest.mark.parametrize("L", [128, 256, 384, 512, 640, 768, 896, 1024])
@pytest.mark.parametrize("T", [130, 512, 998, 1024])
def test_aa_fast_path_sweep(L, T):
    """Every (E, MR) instantiation of the wave-per-stream kernel against the oracle on the same
    complex64 samples; the dispatch is asserted to be the fast path."""
    plan = _lib.lib().ofs_aa_plan(_lib.C64, _lib.FP32, 1, T, L)
    assert plan >= 1000, plan
    rng = np.random.default_rng(L * 7 + T)
    B = 9
    x = (rng.standard_normal((B, 1, T)) + 1j * rng.standard_normal((B, 1, T))) * 0.3
    for b in range(B):                      # [A][A] bursts at random offsets, some streams quiet
        if b % 3 == 2 or T < 2 * L:
            continue
        s = int(rng.integers(0, T - 2 * L + 1))
        a = rng.standard_normal(L) + 1j * rng.standard_normal(L)
        x[b, 0, s:s + L] += a
        x[b, 0, s + L:s + 2 * L] += a
    x = x.astype(np.complex64)
    out = sync_aa.aa_detect_streaming_batched(torch.from_numpy(x).cuda(), L=L, threshold=0.3, hysteresis=32)
    check_fp32_batch(out, x, L, 0.3, 32)


@pytest.mark.parametrize("na", [1, 2])
@pytest.mark.parametrize("L", [128, 256, 512, 1024])
@pytest.mark.parametrize("T", [1025, 1536, 2047, 4096, 5315])
def test_aa_stream_path_sweep(T, L, na):
    """Streaming wave-per-stream kernel (any T, odd T included: 8-byte-aligned stream bases)
    against the oracle; the T = 4096 case is SURVEY §8d's sensitivity shape, T = 5315 x 2
    antennas the reference's own detector input length (sync_aa.py:699-738)."""
    plan = _lib.lib().ofs_aa_plan(_lib.C64, _lib.FP32, na, T, L)
    assert plan >= 1100, plan
    rng = np.random.default_rng(T * 3 + L + na)
    B = 7
    x = (rng.standard_normal((B, na, T)) + 1j * rng.standard_normal((B, na, T))) * 0.3
    for b in range(B):
        if b % 3 == 2 or T < 2 * L:
            continue
        for _ in range(2):
            s = int(rng.integers(0, T - 2 * L + 1))
            a = rng.standard_normal((na, L)) + 1j * rng.standard_normal((na, L))
            x[b, :, s:s + L] += a
            x[b, :, s + L:s + 2 * L] += a
    x = x.astype(np.complex64)
    out = sync_aa.aa_detect_streaming_batched(torch.from_numpy(x).cuda(), L=L, threshold=0.3, hysteresis=32)
    check_fp32_batch(out, x, L, 0.3, 32)
    det = sync_aa.aa_detect_streaming_batched(torch.from_numpy(x).cuda(), L=L, threshold=0.3, hysteresis=32,
                                              outputs=())                # detect-only instantiation
    assert torch.equal(det.n_events, out.n_events)
    for b in range(B):
        n = int(out.n_events[b])
        assert torch.equal(det.ev_int[b, :n], out.ev_int[b, :n])


def test_aa_fast_path_is_used_for_the_benchmark_shape():
    assert _lib.lib().ofs_aa_plan(_lib.C64, _lib.FP32, 1, 1024, 512) >= 1000
    assert _lib.lib().ofs_aa_plan(_lib.C128, _lib.FP64, 1, 1024, 512) == 3024      # fp64 wave-per-stream
    assert _lib.lib().ofs_aa_plan(_lib.C128, _lib.FP64, 1, 9000, 512) == 3024      # any T (fp64 prefix)
    assert _lib.lib().ofs_aa_plan(_lib.C64, _lib.FP32, 1, 4096, 512) == 1124       # streaming fast path
    assert _lib.lib().ofs_aa_plan(_lib.C64, _lib.FP32, 1, 100, 100) in (1, 2)      # L % 128: general engine


# ------------------------------------------------------ receiver back-end ------------
@pytest.mark.parametrize("name", cases("backend"))
def test_receiver_backend_vs_reference_golden(name):
    """sc.run_simulation's back-end chain (sc.py:274-311) on reference-built frames: CFO,
    channel estimate, aligned constellation and EVM within 1e-9 relative; STO / slope 1e-9."""
    d = G(name)
    kw = dict(n_fft=int(d["n_fft"]), cp_len=int(d["cp"]), fs_hz=float(d["fs"]))
    r = core.receiver_backend(d["x"], int(d["pilot_start"]), int(d["data_start"]), d["pilot_used"],
                              d["data_used"], **kw)
    assert abs(r["cfo"] - float(d["cfo"])) < 1e-7
    assert relerr(r["h"], d["h"]) < 1e-9
    assert relerr(r["xa"], d["xa"]) < 1e-9
    assert abs(r["gain"] - complex(d["gain"])) < 1e-9 * max(1.0, abs(complex(d["gain"])))
    assert abs(r["evm"] - float(d["evm"])) < 1e-9 * max(1.0, float(d["evm"]))
    assert abs(r["evm_db"] - float(d["evm_db"])) < 1e-7
    assert abs(r["slope"] - float(d["slope"])) < 1e-9
    assert abs(r["sto"] - float(d["sto"])) < 1e-6
    # given-CFO path and a batch (one frame per row, per-frame known symbols)
    rg = core.receiver_backend(d["x"], int(d["pilot_start"]), int(d["data_start"]), d["pilot_used"],
                               d["data_used"], cfo_hz=float(d["cfo"]), **kw)
    assert relerr(rg["h"], d["h"]) < 1e-9
    xb = torch.from_numpy(np.stack([d["x"]] * 3)).cuda()
    out = core.receiver_backend_batched(xb, [int(d["pilot_start"])] * 3, [int(d["data_start"])] * 3,
                                        np.stack([d["pilot_used"]] * 3), d["data_used"], **kw)
    assert relerr(out["xa"].cpu().numpy()[2], d["xa"]) < 1e-9
    assert np.allclose(out["evm"].cpu().numpy(), float(d["evm"]), rtol=1e-9)


@pytest.mark.parametrize("fmt,nb,N", [("c64", 1, 2048), ("int16", 2, 1024), ("c128", 3, 256), ("c64", 2, 4096),
                                      ("c128", 2, 2048)])
def test_receiver_backend_batched_vs_oracle(fmt, nb, N, variant):
    """The fused back-end (fast kernel for N = 1024 / 2048 / 4096 and 1-2 branches, the generic one
    otherwise and under variant BE_FAST=0) against the oracle's chain, per frame."""
    rng = np.random.default_rng(N + nb)
    B, cp = 6, N // 4
    k = core.centered_subcarrier_indices(N // 2)
    T = 2 * (N + cp) + 400
    x = (rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))) * 300
    x = np.round(x)
    ps = rng.integers(0, 100, B)
    ds = ps + N + cp
    pil = np.exp(2j * np.pi * rng.random((B, k.size)))
    dat = np.exp(2j * np.pi * rng.random(k.size))
    if fmt == "int16":
        xd = torch.from_numpy(np.stack([x.real, x.imag], -1).astype(np.int16)).cuda()
    else:
        xd = torch.from_numpy(x.astype(np.complex64 if fmt == "c64" else np.complex128)).cuda()
    out = core.receiver_backend_batched(xd, ps, ds, pil, dat, n_fft=N, cp_len=cp, fs_hz=1e6, bins=k)
    variant("BE_FAST", 0)
    gen = core.receiver_backend_batched(xd, ps, ds, pil, dat, n_fft=N, cp_len=cp, fs_hz=1e6, bins=k)
    variant("BE_FAST", None)
    for b in range(B):
        r = O.rx_backend(x[b], int(ps[b]), int(ds[b]), N, cp, 1e6, k, pil[b], dat)
        for o in (out, gen):
            assert abs(o["cfo"][b].item() - r["cfo"]) < 1e-6
            assert relerr(o["h"][b].cpu().numpy(), r["h"]) < 1e-9
            assert relerr(o["xa"][b].cpu().numpy(), r["xa"]) < 1e-8
            assert abs(o["evm"][b].item() - r["evm"]) < 1e-8 * max(1.0, r["evm"])
            assert abs(o["slope"][b].item() - r["slope"]) < 1e-9 * max(1.0, abs(r["slope"]))


@pytest.mark.parametrize("T,L", [(1024, 512), (1024, 128), (768, 256)])
def test_aa_fp32_fast_path_two_antennas(T, L):
    """Register-staged fast kernel with two antennas (products and energies summed over the
    antennas, sync_aa.py:463-480): metric within 1e-6, events as the fp32 single-antenna path."""
    assert _lib.lib().ofs_aa_plan(_lib.C64, _lib.FP32, 2, T, L) >= 1000
    rng = np.random.default_rng(T + L)
    B = 24
    x = (rng.standard_normal((B, 2, T)) + 1j * rng.standard_normal((B, 2, T))) * 0.5
    for b in range(0, B, 2):
        s = int(rng.integers(0, T - 2 * L + 1))
        a = rng.standard_normal((2, L)) + 1j * rng.standard_normal((2, L))
        x[b, :, s:s + L] += 2 * a
        x[b, :, s + L:s + 2 * L] += 2 * a
    x = x.astype(np.complex64)
    out = sync_aa.aa_detect_streaming_batched(torch.from_numpy(x).cuda(), L=L, precision="fp32")
    check_fp32_batch(out, x, L)


@pytest.mark.parametrize("N,U", [(1024, 600), (2048, 1200), (4096, 2400)])
def test_receiver_backend_fast_kernel_repeatable_at_full_occupancy(N, U):
    """The fast back-end overlays its phases and reduction slots on the sample buffer (40 KB LDS,
    4-5 workgroups per CU): a cross-wave LDS ordering slip would show as run-to-run differences.
    Enough frames to fill every CU several times, used bins up to the buffer's end (centered
    subcarriers include k = -1), five calls bit for bit."""
    rng = np.random.default_rng(N)
    B, nb, cp = 4096, 2, min(N // 4, 512)
    T = 2 * (N + cp) + 64
    x = torch.from_numpy(((rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))) * 100)
                         .astype(np.complex64)).cuda()
    k = core.centered_subcarrier_indices(U)
    ps = rng.integers(0, 60, B)
    ds = ps + N + cp
    pil = np.exp(2j * np.pi * rng.random((B, k.size)))
    dat = np.exp(2j * np.pi * rng.random(k.size))
    runs = [core.receiver_backend_batched(x, ps, ds, pil, dat, n_fft=N, cp_len=cp, fs_hz=1e6, bins=k)
            for _ in range(5)]
    for r in runs[1:]:
        for key in ("cfo", "h", "xa", "evm", "slope"):
            a, b = runs[0][key], r[key]
            a = torch.view_as_real(a) if a.is_complex() else a
            b = torch.view_as_real(b) if b.is_complex() else b
            assert torch.equal(a.view(torch.int64), b.view(torch.int64)), key
