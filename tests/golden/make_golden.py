"""Generate golden input/output fixtures from the reference (amcolex/ofdm-sync-math).

TEST INFRASTRUCTURE ONLY.  This script imports the read-only reference checkout at
``/root/reference`` (pure Python/NumPy) and runs its hot-path functions on seeded
inputs, writing *data* (inputs + expected outputs) to ``tests/golden/*.npz``.  The
reference itself never leaves this container; only these vectors travel.

Run (from anywhere):
    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py

Reference entry points exercised (file:line into /root/reference):
  sync_aa.aa_detect_streaming          sync_aa.py:421-571
  sc.sc_streaming_metric               sc.py:42-78        (sc.N_FFT overridden per case)
  combined_sc_min.schmidl_cox_streaming_metric  combined_sc_min.py:116-164
  combined_sc_min.minn_streaming_metric         combined_sc_min.py:60-113
  minn.minn_streaming_metric_parameterized      minn.py:697-751
  minn_rtl.minn_rtl_streaming_metric  minn_rtl.py:667-733
  minn_rtl.detect_minn_rtl             minn_rtl.py:750-825
  core.estimate_cfo_from_cp            core.py:179-196
  core.apply_cfo / ofdm_fft_used / ls_channel_estimate / equalize / remove_common_phase /
  align_complex_gain / evm_rms_db / estimate_timing_offset_from_phase_slope
                                       core.py:123-138, 171-176, 339-370, 443-469
  sync_aa.quantize_adc                 sync_aa.py:263-291
  park.park_streaming_metric           park.py:64-114     (park.N_FFT overridden per case)
  zc_freq.compute_frequency_metric     zc_freq.py:62-99   (zc_freq.N_FFT / CYCLIC_PREFIX overridden)
  zc_v2.matched_filter_correlation / normalize_correlation / zc_streaming_detection /
  detect_zc_peaks / detect_zc_preamble zc_v2.py:244-519
  zc.py:106-126 inline combined matched filter (restated in gen_zc from the reference's lines)
Input builders used only to synthesise realistic streams (not part of the parity surface):
  sync_aa.build_aa_preamble / apply_channel_multi_antenna / apply_cfo / quantize_adc,
  sc.build_sc_preamble, combined_sc_min.build_minn_preamble, minn_rtl.build_minn_preamble_generic,
  channel.apply_channel / load_measured_cir, core.build_random_qpsk_symbol / apply_cfo.
"""
from __future__ import annotations

import os
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def _import_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(REF))
    os.chdir(tempfile.mkdtemp(prefix="ofs_golden_"))  # scripts write plots/ relative to cwd
    import core, channel, sc, minn, minn_rtl, combined_sc_min, sync_aa  # noqa: E401
    import park, zc, zc_freq, zc_v2  # noqa: E401
    return dict(core=core, channel=channel, sc=sc, minn=minn, minn_rtl=minn_rtl,
                combined=combined_sc_min, sync_aa=sync_aa, park=park, zc=zc, zc_freq=zc_freq,
                zc_v2=zc_v2)


def _events_aa(res):
    ev = res.events
    ints = np.array([[e.peak_index, e.gate_start, e.gate_end, e.frame_start] for e in ev],
                    dtype=np.int64).reshape(-1, 4)
    reals = np.array([[e.P_at_peak.real, e.P_at_peak.imag, e.M_at_peak, e.cfo_hz] for e in ev],
                     dtype=np.float64).reshape(-1, 4)
    return ints, reals


def gen_aa(R, cases):
    sa = R["sync_aa"]
    pre1024 = sa.build_aa_preamble(1024)[0]
    tx = np.concatenate([np.zeros(500, complex), pre1024, np.zeros(500, complex)])
    # (1) the exact docs/detector_test_vector.csv input, and (2) its CFO variant
    for name, x in (("aa_clean_L512", tx), ("aa_cfo_L512", sa.apply_cfo(tx, 500.0, 15.36e6))):
        res = sa.aa_detect_streaming(x, L=512)
        cases[name] = _aa_case(x[np.newaxis, :], 512, res)

    # (3) run_single_test-shaped inputs (sync_aa.py:669-740): channel + CFO + 12-bit ADC, 2 RX
    grid = [(1024, None, 10.0, 1.0), (1024, "cir1", 0.0, 0.5), (512, "cir2", 5.0, 2.0),
            (256, "cir1", 0.0, 1.0)]
    for plen, ch, snr, fsr in grid:
        rng = np.random.default_rng(42)
        L = plen // 2
        pre = sa.build_aa_preamble(plen)[0]
        pil, _ = sa.build_random_qpsk_symbol(rng)
        dat, _ = sa.build_random_qpsk_symbol(rng)
        txg = np.concatenate([np.zeros(500, complex), pre, pil, dat, np.zeros(500, complex)])
        rx, _, _ = sa.apply_channel_multi_antenna(txg, snr, rng, ch, num_rx_antennas=2)
        rx = sa.apply_cfo(rx, 500.0, sa.SAMPLE_RATE_HZ)
        fs = np.sqrt(np.mean(np.abs(rx) ** 2)) * fsr
        rxq = np.stack([sa.quantize_adc(rx[a], fs) for a in range(2)])
        res = sa.aa_detect_streaming(rxq, L=L)
        cases[f"aa_grid_len{plen}_{ch or 'awgn'}_snr{int(snr)}_fs{fsr}"] = _aa_case(rxq, L, res)

    # (4) integer (int12) inputs, L=128 (BASELINE cfg2 shape): float64 reference on integer values
    rng = np.random.default_rng(7)
    pre = sa.build_aa_preamble(256)[0]
    pil, _ = sa.build_random_qpsk_symbol(rng)
    txg = np.concatenate([np.zeros(300, complex), pre, pil, np.zeros(200, complex)])
    rx, _, _ = sa.apply_channel_multi_antenna(txg, 10.0, rng, "cir1", num_rx_antennas=2)
    rx = rx[:, :1024]
    scale = 2046.0 / np.max(np.abs(np.concatenate([rx.real.ravel(), rx.imag.ravel()])))
    xi = np.clip(np.round(rx.real * scale), -2048, 2047) + 1j * np.clip(np.round(rx.imag * scale), -2048, 2047)
    res = sa.aa_detect_streaming(xi, L=128)
    cases["aa_int12_L128"] = _aa_case(xi, 128, res)

    # (5) edge lengths: T < L, T == L, T == 2L-1, T == 2L, tiny L; random data, 1 and 3 antennas
    rng = np.random.default_rng(11)
    for T, L, na in ((5, 8, 1), (8, 8, 1), (15, 8, 2), (16, 8, 3), (40, 1, 1), (33, 2, 2)):
        x = rng.standard_normal((na, T)) + 1j * rng.standard_normal((na, T))
        res = sa.aa_detect_streaming(x, L=L, threshold=0.1, hysteresis=3)
        c = _aa_case(x, L, res)
        c["threshold"] = np.float64(0.1)
        c["hysteresis"] = np.int64(3)
        cases[f"aa_edge_T{T}_L{L}_a{na}"] = c


def _aa_case(x, L, res):
    ints, reals = _events_aa(res)
    st = res.state
    return dict(kind="aa", x=np.asarray(x, np.complex128), L=np.int64(L), P=st.P, R=st.R, M=st.M,
                valid=st.valid, ev_int=ints, ev_real=reals,
                threshold=np.float64(0.15), hysteresis=np.int64(128), sample_rate=np.float64(15.36e6))


def gen_sc(R, cases):
    sc = R["sc"]
    core = R["core"]
    ch = R["channel"]
    # cfg1: N=64, CP=16, SNR=20 dB, one AWGN burst.  build_sc_preamble is hard-wired to 1200
    # tones (core.py:7), so the N=64 burst is built here: BPSK on even bins within +-30.
    rng = np.random.default_rng(2026)
    N, CP = 64, 16
    idx = np.arange(-30, 31)
    idx = idx[(idx % 2 == 0) & (idx != 0)]
    spec = np.zeros(N, complex)
    spec[(N // 2 + idx) % N] = rng.choice([-1.0, 1.0], size=idx.size)
    sym = np.fft.ifft(np.fft.ifftshift(spec))
    sym /= np.sqrt(np.mean(np.abs(sym) ** 2))
    burst = np.concatenate([np.zeros(100, complex), sym[-CP:], sym, np.zeros(100, complex)])
    rx = ch.apply_channel(burst, 20.0, rng)
    _sc_run(sc, rx, 64, "sc_N64_cfg1", cases)

    # N=1024 and N=2048 on sc.run_simulation-shaped streams (sc.py:159-205), truncated
    rng = np.random.default_rng(0)
    pre = sc.build_sc_preamble(rng, include_cp=True)      # N_FFT=2048 preamble
    pil, _ = core.build_random_qpsk_symbol(rng, include_cp=True)
    tx = np.concatenate([np.zeros(1337, complex), pre, pil])
    cir = ch.load_measured_cir("cir1")[1:2]
    rx = core.apply_cfo(ch.apply_channel(tx, 10.0, rng, cir), 1000.0, core.SAMPLE_RATE_HZ)
    _sc_run(sc, rx[:, :7000], 2048, "sc_N2048_cir1", cases)
    rx2 = ch.apply_channel(tx[:5000], 5.0, np.random.default_rng(5), ch.load_measured_cir("cir2"))
    _sc_run(sc, rx2, 1024, "sc_N1024_cir2_2br", cases)
    # degenerate: T < N (empty outputs) and T == N (one output)
    _sc_run(sc, rx2[:, :100], 128, "sc_short_empty", cases)
    _sc_run(sc, rx2[:, :128], 128, "sc_exact_one", cases)


def _sc_run(sc, rx, N, name, cases):
    old = sc.N_FFT
    sc.N_FFT = N
    try:
        M, P, Rr = sc.sc_streaming_metric(rx)
    finally:
        sc.N_FFT = old
    cases[name] = dict(kind="sc", x=np.atleast_2d(np.asarray(rx, np.complex128)), N=np.int64(N),
                       M=M, P=P, R=Rr)


def gen_combined(R, cases):
    cb = R["combined"]
    mn = R["minn"]
    core = R["core"]
    ch = R["channel"]
    rng = np.random.default_rng(0)
    pre = cb.build_minn_preamble(rng, include_cp=True)
    pil, _ = core.build_random_qpsk_symbol(rng, include_cp=True)
    tx = np.concatenate([np.zeros(1337, complex), pre, pil])
    rx = core.apply_cfo(ch.apply_channel(tx, 10.0, rng, ch.load_measured_cir("cir1")[:2]),
                        1000.0, core.SAMPLE_RATE_HZ)[:, :6500]
    M, P, Rr = cb.schmidl_cox_streaming_metric(rx)
    cases["comb_sc_N2048_cir1_2br"] = dict(kind="comb_sc", x=rx, N=np.int64(2048), M=M, P=P, R=Rr)
    M, P, Rr = cb.schmidl_cox_streaming_metric(rx[:, :3000], symbol_len=256)
    cases["comb_sc_N256"] = dict(kind="comb_sc", x=rx[:, :3000], N=np.int64(256), M=M, P=P, R=Rr)
    M, P, Rr = cb.minn_streaming_metric(rx)
    cases["comb_minn_N2048_cir1_2br"] = dict(kind="minn", x=rx, N=np.int64(2048), M=M, P=P, R=Rr)
    for N in (256, 258, 512):
        M, P, Rr = mn.minn_streaming_metric_parameterized(rx[0, :3000], N)
        cases[f"minn_param_N{N}"] = dict(kind="minn", x=rx[:1, :3000], N=np.int64(N), M=M, P=P, R=Rr)


def _rtl_case(R, x, Q, shift, thr, frac, hyst, toff):
    mr = R["minn_rtl"]
    st = mr.minn_rtl_streaming_metric(x, smooth_shift=shift, threshold_value=thr,
                                      threshold_frac_bits=frac, quarter_len=Q)
    det = mr.detect_minn_rtl(st, hysteresis=hyst, timing_offset=toff)
    ev = np.array([[e.peak_index, e.detected_index, e.gate_segment[0], e.gate_segment[1]]
                   for e in det.events], dtype=np.int64).reshape(-1, 4)
    seg = np.array(det.gate_segments, dtype=np.int64).reshape(-1, 2)
    return dict(kind="minn_rtl", x=np.atleast_2d(np.asarray(x, np.complex128)), Q=np.int64(Q),
                smooth_shift=np.int64(shift), threshold_value=np.int64(thr),
                threshold_frac_bits=np.int64(frac), hysteresis=np.int64(hyst),
                timing_offset=np.int64(toff),
                corr_total=st.corr_total, corr_positive=st.corr_positive,
                smooth_metric=st.smooth_metric, energy_total=st.energy_total,
                corr_scaled=st.corr_scaled, energy_scaled=st.energy_scaled,
                metric_valid=st.metric_valid, above_threshold=st.above_threshold,
                events=ev, gate_segments=seg, gate_mask=det.gate_mask)


def gen_minn_rtl(R, cases):
    mr = R["minn_rtl"]
    core = R["core"]
    ch = R["channel"]
    thr = int(0.10 * (1 << 15))
    for Q, T, seed in ((64, 1024, 3), (512, 6000, 4)):
        rng = np.random.default_rng(seed)
        pre = mr.build_minn_preamble_generic("qpsk_freq", rng, Q=Q)
        pil, _ = core.build_random_qpsk_symbol(rng, include_cp=True)
        tx = np.concatenate([np.zeros(3 * Q, complex), pre, pil])
        rx = ch.apply_channel(tx, 10.0, rng, ch.load_measured_cir("cir1")[:2])[:, :T]
        # 12-bit quantisation in the style of ref/test_minn_preamble_detector.py:150-161
        s = 2046.0 / np.max(np.abs(np.concatenate([rx.real.ravel(), rx.imag.ravel()])))
        xi = np.clip(np.round(rx.real * s), -2048, 2047) + 1j * np.clip(np.round(rx.imag * s), -2048, 2047)
        cases[f"rtl_Q{Q}_int12"] = _rtl_case(R, xi, Q, 3, thr, 15, 2, 0)
        if Q == 64:
            cases["rtl_Q64_float"] = _rtl_case(R, rx, Q, 3, thr, 15, 2, 0)
            cases["rtl_Q64_int12_noshift_h0"] = _rtl_case(R, xi, Q, 0, thr, 15, 0, -5)
            cases["rtl_Q64_int12_thr0_h5"] = _rtl_case(R, xi[:1], Q, 2, 0, 15, 5, 7)


def gen_cp_cfo(R, cases):
    core = R["core"]
    ch = R["channel"]
    rng = np.random.default_rng(9)
    sym, _ = core.build_random_qpsk_symbol(rng, include_cp=True)
    tx = np.concatenate([np.zeros(200, complex), sym, sym])
    rx = core.apply_cfo(ch.apply_channel(tx, 15.0, rng, ch.load_measured_cir("cir1")[:2]),
                        1234.5, core.SAMPLE_RATE_HZ)
    starts = np.array([0, 200, 250, 333, 1000], dtype=np.int64)
    cfo = np.array([core.estimate_cfo_from_cp(rx, int(s), 2048, 512, core.SAMPLE_RATE_HZ)
                    for s in starts])
    cfo1 = np.array([core.estimate_cfo_from_cp(rx[0], int(s), 2048, 256, 15.36e6) for s in starts])
    cases["cp_cfo"] = dict(kind="cp_cfo", x=rx, starts=starts, n_fft=np.int64(2048),
                           cp_len=np.int64(512), fs=np.float64(core.SAMPLE_RATE_HZ), cfo=cfo,
                           cfo_1br_cp256=cfo1, fs_1br=np.float64(15.36e6))
    # CP searches around an estimated start (core.py:199-336): estimates early / late / near the
    # edges (empty range -> fallback), default and explicit span / win_len, 1 and 2 branches
    est = np.array([0, 150, 200, 260, 1000, rx.shape[1] - 2048 - 512 - 3, rx.shape[1] - 2048 - 512], np.int64)
    fs = core.SAMPLE_RATE_HZ
    srch = dict(kind="cp_search", x=rx, est=est, n_fft=np.int64(2048), cp_len=np.int64(512),
                fs=np.float64(fs))
    srch["robust"] = np.array([core.estimate_cfo_from_cp_robust(rx, int(e), 2048, 512, fs) for e in est])
    srch["robust_s40_w100"] = np.array([core.estimate_cfo_from_cp_robust(rx, int(e), 2048, 512, fs, span=40,
                                                                          win_len=100) for e in est])
    srch["robust_1br_s0"] = np.array([core.estimate_cfo_from_cp_robust(rx[0], int(e), 2048, 512, fs, span=0)
                                      for e in est])
    pk = [core.estimate_cfo_from_cp_peak_with_index(rx, int(e), 2048, 512, fs) for e in est]
    srch["peak_cfo"] = np.array([p[0] for p in pk])
    srch["peak_d"] = np.array([p[1] for p in pk], np.int64)
    srch["peak_only"] = np.array([core.estimate_cfo_from_cp_peak(rx, int(e), 2048, 512, fs) for e in est])
    pk = [core.estimate_cfo_from_cp_peak_with_index(rx[1], int(e), 2048, 256, fs, span=300) for e in est]
    srch["peak_1br_s300_cfo"] = np.array([p[0] for p in pk])
    srch["peak_1br_s300_d"] = np.array([p[1] for p in pk], np.int64)
    srch["find_start"] = np.array([core.find_cp_start_via_corr(rx, int(e), 2048, 512) for e in est], np.int64)
    srch["find_start_h64"] = np.array([core.find_cp_start_via_corr(rx, int(e), 2048, 512, search_half=64)
                                       for e in est], np.int64)
    cases["cp_search"] = srch


def gen_backend(R, cases):
    """Receiver back-end chain of sc.run_simulation (sc.py:274-311), run with the reference's
    own core.py helpers on frames built by its builders; the pilot/data CP starts are the true
    ones shifted by a few samples (the detector's job is upstream)."""
    core, ch = R["core"], R["channel"]
    N, CP, fs = core.N_FFT, core.CYCLIC_PREFIX, core.SAMPLE_RATE_HZ
    k = core.centered_subcarrier_indices(core.NUM_ACTIVE_SUBCARRIERS)
    for name, seed, snr, cir, cfo, shift in (("backend_cir1_2br", 21, 15.0, "cir1", 1000.0, 3),
                                             ("backend_awgn_1br", 22, 20.0, None, -2500.0, 0),
                                             ("backend_cir2_2br_early", 23, 10.0, "cir2", 700.0, -4)):
        rng = np.random.default_rng(seed)
        pil, pil_used = core.build_random_qpsk_symbol(rng, include_cp=True)
        dat, dat_used = core.build_random_qpsk_symbol(rng, include_cp=True)
        pad = 600
        tx = np.concatenate([np.zeros(pad, complex), pil, dat, np.zeros(300, complex)])
        rx = ch.apply_channel(tx, snr, rng, None if cir is None else ch.load_measured_cir(cir)[:2])
        rx = core.apply_cfo(rx, cfo, fs)
        ps = pad + shift
        ds = ps + CP + N
        cfo_est = core.estimate_cfo_from_cp(rx, ps, N, CP, fs)        # sc.py:278-284
        rxc = core.apply_cfo(rx, -cfo_est, fs)                         # sc.py:286
        eff = rxc if rxc.ndim == 1 else np.mean(rxc, axis=0)           # sc.py:289
        y_p = core.ofdm_fft_used(eff[ps + CP:ps + CP + N])
        h = core.ls_channel_estimate(y_p, pil_used)
        slope, sto = core.estimate_timing_offset_from_phase_slope(h)
        y_d = core.ofdm_fft_used(eff[ds + CP:ds + CP + N])
        xhat = core.equalize(y_d, h)
        xa, gain = core.align_complex_gain(xhat, dat_used)
        evm, evm_db = core.evm_rms_db(xa, dat_used)
        cases[name] = dict(kind="backend", x=np.atleast_2d(rx), pilot_start=np.int64(ps), data_start=np.int64(ds),
                           n_fft=np.int64(N), cp=np.int64(CP), fs=np.float64(fs), bins=k.astype(np.int64),
                           pilot_used=pil_used, data_used=dat_used, cfo=np.float64(cfo_est), h=h, xa=xa,
                           gain=np.complex128(gain), evm=np.float64(evm), evm_db=np.float64(evm_db),
                           slope=np.float64(slope), sto=np.float64(sto), y_pilot=y_p)


def gen_backend_ops(R, cases):
    """The back-end helpers one by one, as sc.run_simulation calls them (sc.py:274-311), plus
    core.apply_cfo and sync_aa.quantize_adc: inputs and the reference's outputs per helper."""
    core, ch, sa = R["core"], R["channel"], R["sync_aa"]
    N, CP, fs = core.N_FFT, core.CYCLIC_PREFIX, core.SAMPLE_RATE_HZ
    for name, seed, snr, cir, cfo, shift in (("bops_cir1_2br", 31, 12.0, "cir1", 1500.0, 2),
                                             ("bops_awgn_1br", 32, 25.0, None, -800.0, 0)):
        rng = np.random.default_rng(seed)
        pil, pil_used = core.build_random_qpsk_symbol(rng, include_cp=True)
        dat, dat_used = core.build_random_qpsk_symbol(rng, include_cp=True)
        pad = 400
        tx = np.concatenate([np.zeros(pad, complex), pil, dat, np.zeros(200, complex)])
        rx = ch.apply_channel(tx, snr, rng, None if cir is None else ch.load_measured_cir(cir)[:2])
        rx_cfo = core.apply_cfo(rx, cfo, fs)                               # core.py:123-138 (1-D or 2-D)
        rx1_cfo = core.apply_cfo(np.atleast_2d(rx)[0], -cfo / 3, fs)
        ps = pad + shift
        ds = ps + CP + N
        eff = np.mean(np.atleast_2d(core.apply_cfo(rx_cfo, -cfo, fs)), axis=0)
        sym_p, sym_d = eff[ps + CP:ps + CP + N], eff[ds + CP:ds + CP + N]
        y_p = core.ofdm_fft_used(sym_p)                                   # core.py:171-176
        y_short = core.ofdm_fft_used(sym_p[:N - 300])                     # fft(x, n=N) zero-pads
        y_long = core.ofdm_fft_used(eff[ps:ps + N + 200])                 # ... and truncates
        h = core.ls_channel_estimate(y_p, pil_used)                       # :339-341
        y_d = core.ofdm_fft_used(sym_d)
        xhat = core.equalize(y_d, h)                                      # :344-345
        x_cpe, cpe = core.remove_common_phase(xhat)                       # :348-354, mean angle
        x_cpe_ref, cpe_ref = core.remove_common_phase(xhat, dat_used)     # ... against a reference
        xa, gain = core.align_complex_gain(xhat, dat_used)                # :357-362
        evm, evm_db = core.evm_rms_db(xa, dat_used)                       # :365-370
        slope, sto = core.estimate_timing_offset_from_phase_slope(h)      # :443-469
        rms = float(np.sqrt(np.mean(np.abs(np.atleast_2d(rx_cfo)[0]) ** 2)))
        q64 = sa.quantize_adc(np.atleast_2d(rx_cfo)[0], 4.0 * rms)                         # sync_aa.py:263-291
        q64_np = sa.quantize_adc(np.atleast_2d(rx_cfo)[0], np.float64(2.5 * rms), bits=8)  # numpy scalar
        x32 = np.atleast_2d(rx_cfo)[0].astype(np.complex64)
        q32 = sa.quantize_adc(x32, 3.0 * rms)                                              # fp32 (weak scalar)
        q32_np = sa.quantize_adc(x32, np.float64(3.0 * rms))                              # promotes to fp64
        cases[name] = dict(kind="backend_ops", rx=rx, cfo=np.float64(cfo), fs=np.float64(fs), rx_cfo=rx_cfo,
                           rx1_cfo=rx1_cfo, sym_p=sym_p, sym_d=sym_d, y_p=y_p, y_short=y_short, y_long=y_long,
                           pil_used=pil_used, dat_used=dat_used, h=h, y_d=y_d, xhat=xhat, x_cpe=x_cpe,
                           cpe=np.float64(cpe), x_cpe_ref=x_cpe_ref, cpe_ref=np.float64(cpe_ref), xa=xa,
                           gain=np.complex128(gain), evm=np.float64(evm), evm_db=np.float64(evm_db),
                           slope=np.float64(slope), sto=np.float64(sto), rms=np.float64(rms), q64=q64,
                           q64_np=q64_np, x32=x32, q32=q32, q32_np=q32_np)


def gen_park(R, cases):
    pk = R["park"]
    core = R["core"]
    ch = R["channel"]
    for N, T, seed in ((2048, 7000, 0), (256, 3000, 1), (64, 400, 2)):
        old = pk.N_FFT
        pk.N_FFT = N
        try:
            rng = np.random.default_rng(seed)
            if N == 2048:
                pre = pk.build_park_preamble(rng, include_cp=True)
                tx = np.concatenate([np.zeros(1337, complex), pre, core.build_random_qpsk_symbol(rng)[0]])
                rx = ch.apply_channel(tx, 10.0, rng, ch.load_measured_cir("cir1")[:2])[:, :T]
            else:
                rx = rng.standard_normal((2, T)) + 1j * rng.standard_normal((2, T))
                h = N // 2
                a = rng.standard_normal(h) + 1j * rng.standard_normal(h)
                rx[:, 100:100 + h] += a[::-1] * 2          # symmetric structure around d = 100 + h
                rx[:, 100 + h:100 + 2 * h] += a * 2
            ds, M, P, E = pk.park_streaming_metric(rx)
        finally:
            pk.N_FFT = old
        cases[f"park_N{N}"] = dict(kind="park", x=rx, N=np.int64(N), ds=ds, M=M, P=P, E=E)


def gen_zc(R, cases):
    zf = R["zc_freq"]
    z2 = R["zc_v2"]
    zc = R["zc"]
    core = R["core"]
    ch = R["channel"]
    # zc_freq.compute_frequency_metric (zc_freq.py:62-99); N_FFT / CYCLIC_PREFIX read at call time
    for N, CP, T, seed in ((2048, 512, 4200, 0), (256, 64, 1500, 3)):
        oldN, oldC = zf.N_FFT, zf.CYCLIC_PREFIX
        zf.N_FFT, zf.CYCLIC_PREFIX = N, CP
        try:
            rng = np.random.default_rng(seed)
            if N == 2048:
                tx = np.concatenate([np.zeros(1337, complex), zf.build_pss_symbol(include_cp=True)])
                rx = ch.apply_channel(tx, 10.0, rng, ch.load_measured_cir("cir1")[:2])[:, :T]
            else:
                rx = rng.standard_normal((2, T)) + 1j * rng.standard_normal((2, T))
            bins, tmpl, energy = zf.make_pss_frequency_template()
            metric = zf.compute_frequency_metric(rx, bins, tmpl, energy)
        finally:
            zf.N_FFT, zf.CYCLIC_PREFIX = oldN, oldC
        cases[f"zcfreq_N{N}"] = dict(kind="zc_freq", x=rx, N=np.int64(N), CP=np.int64(CP), bins=bins,
                                     template=tmpl, template_energy=np.float64(energy), metric=metric)
    # zc_v2 matched filter / normaliser / streaming detection / gate (zc_v2.py:244-450), and the
    # inline zc.py combined matched filter (zc.py:106-126, restated here statement for statement)
    rng = np.random.default_rng(8)
    ref = z2.build_pss_symbol(include_cp=False)
    tx = np.concatenate([np.zeros(1500, complex), z2.build_pss_symbol(include_cp=True),
                         core.build_random_qpsk_symbol(rng)[0]])
    rx = core.apply_cfo(ch.apply_channel(tx, 10.0, rng, ch.load_measured_cir("cir1")[:2]), 1000.0,
                        core.SAMPLE_RATE_HZ)[:, :6000]
    corr = [z2.matched_filter_correlation(b, ref) for b in rx]
    norm = [z2.normalize_correlation(c, b, ref) for c, b in zip(corr, rx)]
    det = z2.detect_zc_preamble(rx)
    st = det.state
    ev = np.array([[e.peak_index, e.gate_start, e.gate_end, e.detected_start] for e in det.events],
                  dtype=np.int64).reshape(-1, 4)
    evv = np.array([e.peak_value for e in det.events], dtype=np.float64)
    pss_reference = zc.build_pss_symbol(include_cp=False)
    pss_conj = np.conj(pss_reference[::-1])
    reference_norm = np.sqrt(np.sum(np.abs(pss_reference) ** 2))
    window = np.ones(pss_reference.size, dtype=float)
    num = sum(np.convolve(b, pss_conj) for b in rx)
    pw = sum(np.convolve(np.abs(b) ** 2, window) for b in rx)
    combined = num / (reference_norm * np.sqrt(np.maximum(pw, 0.0) + 1e-12))
    cases["zc_mf"] = dict(kind="zc_mf", x=rx, ref=ref, corr=np.stack(corr), norm=np.stack(norm),
                          zc_ref=pss_reference, zc_combined=combined,
                          corr_mag=st.corr_mag, local_sum=st.local_sum, corr_scaled=st.corr_scaled,
                          thresh_scaled=st.thresh_scaled, above_threshold=st.above_threshold,
                          metric_valid=st.metric_valid, events=ev, peak_values=evv,
                          gate_mask=det.gate_mask, window_size=np.int64(z2.CORR_WINDOW_SIZE),
                          thresh_value=np.int64(z2.THRESH_VALUE), thresh_frac_bits=np.int64(z2.THRESH_FRAC_BITS),
                          min_corr_mag=np.float64(z2.MIN_CORR_MAG), hysteresis=np.int64(z2.HYSTERESIS))


def gen_post(R, cases):
    """Detection post-processing on metrics the reference produced above:
    sc.find_plateau_end_from_metric (sc.py:81-146), minn.find_minn_peak (minn.py:131-205),
    minn._trailing_average (minn.py:115-128), combined_sc_min.find_minn_peak (:212-259) with
    _streaming_peak_detector (:183-209), and the S&C gate of combined_sc_min.run_simulation
    (:337-358, inline code restated here statement for statement)."""
    sc, minn, comb = R["sc"], R["minn"], R["combined"]
    rng = np.random.default_rng(11)
    # ---- sc plateau end: reference metrics + shapes that reach the other branches ----
    pl = []
    for name, cp, la, sw in (("sc_N2048_cir1", 512, 128, 16), ("sc_N1024_cir2_2br", 256, 64, 16),
                             ("sc_N64_cfg1", 16, None, 8), ("sc_N2048_cir1", 512, None, 8)):
        pl.append((cases[name]["M"], cp, la, sw))
    ramp = np.linspace(0.0, 1.0, 300)
    spikes = np.zeros(400)
    spikes[::37] = rng.uniform(0.2, 1.0, spikes[::37].size)
    plateau = np.concatenate([np.full(50, 0.1), np.full(120, 0.9), np.full(80, 0.2)])
    pl += [(ramp, 64, None, 8), (spikes, 1, None, 1), (spikes, 3, 2, 4), (np.zeros(100), 16, None, 8),
           (plateau, 40, None, 1), (plateau[::-1].copy(), 1, 5, 1), (rng.random(257), 2, 1, 3),
           (np.array([0.3]), 16, None, 8), (np.array([0.1, 0.5]), 1, None, 1), (np.zeros(0), 16, None, 8)]
    for i, (M, cp, la, sw) in enumerate(pl):
        try:
            out = np.int64(sc.find_plateau_end_from_metric(np.asarray(M, float), cp, lookahead=la, smooth_win=sw))
            err = np.int64(0)
        except ValueError:
            out, err = np.int64(-1), np.int64(1)
        cases[f"post_plateau_{i:02d}"] = dict(kind="plateau", M=np.asarray(M, float), cp=np.int64(cp),
                                              lookahead=np.int64(-1 if la is None else la),
                                              smooth_win=np.int64(sw), index=out, error=err)
    # ---- minn.find_minn_peak ----
    mp = [(cases["comb_minn_N2048_cir1_2br"]["M"], 16, 0.5, None),
          (cases["minn_param_N256"]["M"], 8, 0.5, None),
          (cases["minn_param_N512"]["M"], 16, 0.5, (100, 900)),
          (cases["minn_param_N512"]["M"], 1, 0.7, (2000, 1000)),        # start >= end: whole range
          (cases["comb_minn_N2048_cir1_2br"]["M"], 16, 0.5, (0, 50)),    # bounds miss the gate
          (np.concatenate([rng.random(40) * 0.1, [0.9] * 5, [0.1] * 10, [0.8] * 5, rng.random(30) * 0.1]),
           1, 0.5, None),                                              # two equal runs: earliest wins
          (-np.abs(rng.standard_normal(64)), 4, 0.5, None),              # no positive peak: ValueError
          (np.zeros(0), 4, 0.5, None)]                                   # empty: ValueError
    for i, (M, sw, thr, bnd) in enumerate(mp):
        M = np.asarray(M, float)
        try:
            pk, gate, Ms = minn.find_minn_peak(M, smooth_win=sw, gate_threshold=thr, search_bounds=bnd)
            err = np.int64(0)
        except ValueError:
            pk, gate, Ms, err = -1, np.zeros(M.size, bool), np.zeros(M.size), np.int64(1)
        cases[f"post_minnpeak_{i:02d}"] = dict(
            kind="minn_peak", M=M, smooth_win=np.int64(sw), thr=np.float64(thr),
            bounds=np.array([-1, -1] if bnd is None else bnd, np.int64), peak=np.int64(pk),
            gate=np.asarray(gate, bool), Ms=np.asarray(Ms, float), error=err)
    cases["post_trailing_avg"] = dict(
        kind="trailing", x=np.maximum(cases["comb_minn_N2048_cir1_2br"]["M"], 0.0),
        y16=comb._trailing_average(np.maximum(cases["comb_minn_N2048_cir1_2br"]["M"], 0.0), win=16),
        y1=minn._trailing_average(np.maximum(cases["comb_minn_N2048_cir1_2br"]["M"], 0.0), win=1),
        y3=minn._trailing_average(np.maximum(cases["minn_param_N256"]["M"], 0.0), win=3),
        x3=np.maximum(cases["minn_param_N256"]["M"], 0.0))
    # ---- combined_sc_min back end: S&C gate -> find_minn_peak on the Minn metric ----
    M_sc, M_mn = cases["comb_sc_N2048_cir1_2br"]["M"], cases["comb_minn_N2048_cir1_2br"]["M"]
    max_sc = float(np.max(M_sc))                                        # combined_sc_min.py:340-355
    gate = (M_sc / max_sc >= comb.SC_GATE_THRESHOLD) if max_sc > 0 else (M_sc >= comb.SC_GATE_THRESHOLD)
    if not np.any(gate):
        gate = np.zeros_like(gate, dtype=bool)
        gate[int(np.argmax(M_sc))] = True
    first, last = int(np.argmax(gate)), int(gate.size - np.argmax(gate[::-1]) - 1)
    pk = comb.find_minn_peak(M_mn, smooth_win=comb.SMOOTH_WIN, gate_mask=gate, search_bounds=None)
    cases["post_comb_detect"] = dict(kind="comb_detect", M_sc=M_sc, M_minn=M_mn, gate=gate,
                                     span=np.array([first, last + 1], np.int64), peak=np.int64(pk),
                                     smooth_win=np.int64(comb.SMOOTH_WIN))
    # streaming peak on multi-run masks (first run only), metrics with ties
    met = np.round(rng.random(500) * 8) / 8
    sp = {}
    for j in range(4):
        mask = rng.random(500) < (0.02, 0.2, 0.6, 0.0)[j]
        sp[f"mask{j}"] = mask
        r = comb._streaming_peak_detector(met, mask)
        sp[f"peak{j}"] = np.int64(-1 if r is None else r)
    pk_b = comb.find_minn_peak(M_mn, smooth_win=4, gate_mask=gate, search_bounds=(first + 5, last - 5))
    cases["post_streaming_peak"] = dict(kind="streaming_peak", metric=met, peak_bounded=np.int64(pk_b), **sp)


def gen_synth(R, cases):
    """Input builders the GPU synthesis restates (synth.py / synth.hip): the measured CIR banks
    (channel.load_measured_cir, channel.py:15-48), the [A][A] preambles (sync_aa.build_aa_preamble,
    sync_aa.py:160-235) and random QPSK OFDM symbols (sync_aa.build_random_qpsk_symbol,
    sync_aa.py:238-260), plus one run_single_test frame chain without noise (convolution with the
    CIR bank, sync_aa.py:577-634, and CFO, :637-645)."""
    ch, sa = R["channel"], R["sync_aa"]
    d = {}
    for name in ("cir1", "cir2"):
        d[name] = ch.load_measured_cir(name)
    for ln in sa.PREAMBLE_LENGTHS:
        d[f"pre{ln}"] = sa.build_aa_preamble(ln)[0]
    rng = np.random.default_rng(7)
    syms, qpsk = [], []
    for _ in range(3):
        s_, q_ = sa.build_random_qpsk_symbol(rng)
        syms.append(s_)
        qpsk.append(q_)
    d["qpsk_symbols"], d["qpsk_values"] = np.array(syms), np.array(qpsk)
    frame = np.concatenate([np.zeros(sa.TX_PRE_PAD_SAMPLES, complex), d["pre1024"], syms[0], syms[1],
                            np.zeros(sa.TX_POST_PAD_SAMPLES, complex)])
    cir = d["cir1"][:2]
    rx = np.stack([np.convolve(frame, cir[a]) for a in range(2)])
    d["frame_cir1_cfo500"] = sa.apply_cfo(rx, 500.0, sa.SAMPLE_RATE_HZ)
    d["geometry"] = np.array([sa.N_FFT, sa.CYCLIC_PREFIX, sa.NUM_ACTIVE_SUBCARRIERS, sa.TX_PRE_PAD_SAMPLES,
                              sa.TX_POST_PAD_SAMPLES])
    cases["synth_builders"] = dict(kind="synth", **d)


def main():
    R = _import_reference()
    cases: dict[str, dict] = {}
    gen_aa(R, cases)
    gen_sc(R, cases)
    gen_combined(R, cases)
    gen_minn_rtl(R, cases)
    gen_cp_cfo(R, cases)
    gen_backend(R, cases)
    gen_backend_ops(R, cases)
    gen_park(R, cases)
    gen_zc(R, cases)
    gen_post(R, cases)
    gen_synth(R, cases)
    OUT.mkdir(parents=True, exist_ok=True)
    only = set(sys.argv[1:])               # optional case names: rewrite only those files
    for name, d in cases.items():
        if only and name not in only:
            continue
        arrs = {k: (np.asarray(v) if not isinstance(v, str) else np.array(v)) for k, v in d.items()}
        np.savez_compressed(OUT / f"{name}.npz", **arrs)
    (OUT / "MANIFEST.txt").write_text(
        "Generated by tests/golden/make_golden.py from amcolex/ofdm-sync-math @ /root/reference\n"
        f"numpy {np.__version__}\n" + "\n".join(sorted(cases)) + "\n")
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
