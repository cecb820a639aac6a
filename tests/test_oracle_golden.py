"""CPU: the oracle against the reference's own fixtures and the captured golden vectors,
plus a CPU check of the closed-form (parallel) event formulation used by the HIP kernel."""
import glob
import os
import re

import numpy as np
import pytest

import ofdm_oracle as O
from conftest import GOLDEN

CASES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def _load(path):
    return np.load(path, allow_pickle=False)


def test_fixture_inventory():
    names = {os.path.basename(p)[:-4] for p in CASES}
    assert {"aa_clean_L512", "aa_cfo_L512", "aa_int12_L128", "sc_N64_cfg1",
            "comb_sc_N2048_cir1_2br", "comb_minn_N2048_cir1_2br", "rtl_Q64_int12",
            "rtl_Q512_int12", "cp_cfo"} <= names


@pytest.mark.parametrize("path", CASES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_matches_reference_golden(path):
    d = _load(path)
    kind = str(d["kind"])
    if kind == "aa":
        P, R, M, valid, ei, er = O.aa_detect(d["x"], int(d["L"]), float(d["threshold"]),
                                             int(d["hysteresis"]), float(d["sample_rate"]))
        scale = max(1.0, float(np.abs(d["P"]).max(initial=0)))
        assert np.max(np.abs(P - d["P"]), initial=0) <= 1e-12 * scale
        assert np.max(np.abs(R - d["R"]), initial=0) <= 1e-12 * max(1.0, float(d["R"].max(initial=0)))
        assert np.max(np.abs(M - d["M"]), initial=0) <= 1e-12
        assert np.array_equal(valid, d["valid"])
        assert np.array_equal(ei, d["ev_int"])
        assert np.allclose(er, d["ev_real"], rtol=1e-12, atol=1e-9)
        if "int12" in path:
            # integer inputs: P is an exact integer sum.  R is not: the reference squares
            # np.abs(x) (a rounded hypot, sync_aa.py:479), so it is only ~1 ulp-exact.
            assert np.array_equal(P, d["P"])
            assert np.allclose(R, d["R"], rtol=1e-14, atol=0)
    elif kind in ("sc", "comb_sc", "minn"):
        fn = {"sc": O.sc_metric, "comb_sc": O.comb_sc_metric, "minn": O.minn_metric}[kind]
        M, P, R = fn(d["x"], int(d["N"]))
        assert M.shape == d["M"].shape
        if M.size:
            s = float(np.abs(d["P"]).max())
            assert np.max(np.abs(P - d["P"])) <= 1e-12 * max(s, 1.0) * 1e3
            assert np.max(np.abs(R - d["R"])) <= 1e-12 * float(d["R"].max()) * 1e3
            assert np.max(np.abs(M - d["M"])) <= 1e-10
    elif kind == "minn_rtl":
        s = O.minn_rtl_metric(d["x"], int(d["Q"]), int(d["smooth_shift"]), int(d["threshold_value"]),
                              int(d["threshold_frac_bits"]))
        exact = "int12" in path
        for k, v in s.items():
            if exact:
                assert np.array_equal(v, d[k]), k
            else:
                assert np.allclose(v, d[k], rtol=1e-9, atol=1e-6), k
        ev, seg, mask = O.detect_minn_rtl(s["corr_positive"], s["above_threshold"], s["metric_valid"],
                                          int(d["hysteresis"]), int(d["timing_offset"]))
        assert np.array_equal(ev, d["events"])
        assert np.array_equal(seg, d["gate_segments"])
        assert np.array_equal(mask, d["gate_mask"])
    elif kind == "cp_cfo":
        c = [O.cp_cfo(d["x"], int(s), int(d["n_fft"]), int(d["cp_len"]), float(d["fs"]))[0] for s in d["starts"]]
        assert np.allclose(c, d["cfo"], rtol=0, atol=1e-9)
        c1 = [O.cp_cfo(d["x"][0], int(s), 2048, 256, float(d["fs_1br"]))[0] for s in d["starts"]]
        assert np.allclose(c1, d["cfo_1br_cp256"], rtol=0, atol=1e-9)
    elif kind == "backend":
        r = O.rx_backend(d["x"], int(d["pilot_start"]), int(d["data_start"]), int(d["n_fft"]), int(d["cp"]),
                         float(d["fs"]), d["bins"], d["pilot_used"], d["data_used"])
        assert abs(r["cfo"] - float(d["cfo"])) < 1e-9
        for k in ("h", "xa"):
            assert np.allclose(r[k], d[k], rtol=1e-12, atol=1e-12), k
        for k in ("evm", "evm_db", "slope", "sto"):
            assert abs(r[k] - float(d[k])) < 1e-9, k
        assert abs(r["gain"] - complex(d["gain"])) < 1e-12
    elif kind == "backend_ops":
        k = np.concatenate((np.arange(-600, 0), np.arange(1, 601)))
        np.testing.assert_array_equal(O.apply_cfo(d["rx"], float(d["cfo"]), float(d["fs"])), d["rx_cfo"])
        np.testing.assert_array_equal(O.fft_used(d["sym_p"], 2048, k), d["y_p"])
        np.testing.assert_array_equal(O.fft_used(d["sym_p"][:2048 - 300], 2048, k), d["y_short"])
        np.testing.assert_array_equal(O.cdiv_eps(d["y_p"], d["pil_used"], 1e-9), d["h"])
        np.testing.assert_array_equal(O.cdiv_eps(d["y_d"], d["h"], 1e-9), d["xhat"])
        x, c = O.remove_common_phase(d["xhat"])
        np.testing.assert_array_equal(x, d["x_cpe"])
        assert c == float(d["cpe"])
        x, c = O.remove_common_phase(d["xhat"], d["dat_used"])
        np.testing.assert_array_equal(x, d["x_cpe_ref"])
        assert c == float(d["cpe_ref"])
        xa, g = O.align_complex_gain(d["xhat"], d["dat_used"])
        np.testing.assert_array_equal(xa, d["xa"])
        assert g == complex(d["gain"])
        assert O.evm_rms_db(d["xa"], d["dat_used"]) == (float(d["evm"]), float(d["evm_db"]))
        assert O.phase_slope(d["h"], k, 2048) == (float(d["slope"]), float(d["sto"]))
        x = np.atleast_2d(d["rx_cfo"])[0]
        rms = float(d["rms"])
        np.testing.assert_array_equal(O.quantize_adc(x, 4.0 * rms), d["q64"])
        np.testing.assert_array_equal(O.quantize_adc(x, np.float64(2.5 * rms), 8), d["q64_np"])
        q32 = O.quantize_adc(d["x32"], 3.0 * rms)
        assert q32.dtype == np.complex64
        np.testing.assert_array_equal(q32, d["q32"])
        np.testing.assert_array_equal(O.quantize_adc(d["x32"], np.float64(3.0 * rms)), d["q32_np"])
    elif kind == "cp_search":
        x, N, cp, fs = d["x"], int(d["n_fft"]), int(d["cp_len"]), float(d["fs"])
        est = [int(e) for e in d["est"]]
        close = lambda a, b: np.allclose(a, b, rtol=0, atol=1e-8)   # noqa: E731
        assert close([O.cp_cfo_robust(x, e, N, cp, fs) for e in est], d["robust"])
        assert close([O.cp_cfo_robust(x, e, N, cp, fs, span=40, win_len=100) for e in est], d["robust_s40_w100"])
        assert close([O.cp_cfo_robust(x[0], e, N, cp, fs, span=0) for e in est], d["robust_1br_s0"])
        pk = [O.cp_cfo_peak(x, e, N, cp, fs) for e in est]
        assert close([p[0] for p in pk], d["peak_cfo"]) and close([p[0] for p in pk], d["peak_only"])
        assert [p[1] for p in pk] == list(d["peak_d"])
        pk = [O.cp_cfo_peak(x[1], e, N, 256, fs, span=300) for e in est]
        assert close([p[0] for p in pk], d["peak_1br_s300_cfo"]) and [p[1] for p in pk] == list(d["peak_1br_s300_d"])
        assert [O.find_cp_start(x, e, N, cp) for e in est] == list(d["find_start"])
        assert [O.find_cp_start(x, e, N, cp, search_half=64) for e in est] == list(d["find_start_h64"])
    elif kind == "park":
        ds, M, P, E = O.park_metric(d["x"], int(d["N"]))
        assert np.array_equal(ds, d["ds"])
        assert np.allclose(P, d["P"], rtol=0, atol=1e-11 * float(np.abs(d["P"]).max()))
        assert np.allclose(E, d["E"], rtol=1e-12, atol=0)
        assert np.allclose(M, d["M"], rtol=1e-9, atol=1e-12)
    elif kind == "zc_freq":
        idx, t, et = O.zc_template()
        assert np.array_equal(idx, d["bins"]) and np.allclose(t, d["template"], rtol=0, atol=1e-15)
        assert et == float(d["template_energy"])
        m = O.zc_freq_metric(d["x"], int(d["N"]), int(d["CP"]), idx, t, et)
        assert np.allclose(m, d["metric"], rtol=1e-9, atol=1e-13)
    elif kind == "zc_mf":
        x, ref = d["x"], d["ref"]
        N = ref.size
        assert np.allclose(O.pss_symbol(N), ref, rtol=0, atol=1e-14)
        assert np.allclose(O.pss_symbol(N), d["zc_ref"], rtol=0, atol=1e-14)
        for b in range(x.shape[0]):
            c = O.matched_filter(x[b], ref)
            assert np.allclose(c, d["corr"][b], rtol=0, atol=1e-12)
            assert np.allclose(O.normalize_correlation(c, x[b], ref), d["norm"][b], rtol=0, atol=1e-12)
        assert np.allclose(O.zc_combined(x, ref), d["zc_combined"], rtol=0, atol=1e-12)
        mag = np.abs(d["norm"].sum(axis=0))
        assert np.allclose(mag, d["corr_mag"], rtol=0, atol=1e-15)
        st = O.zc_streaming_detection(d["corr_mag"], int(d["window_size"]), int(d["thresh_value"]),
                                      int(d["thresh_frac_bits"]), float(d["min_corr_mag"]))
        for k in ("local_sum", "corr_scaled", "thresh_scaled", "above_threshold", "metric_valid"):
            assert np.array_equal(st[k], d[k]), k        # literal recursion: bit-identical
        ev, vals, mask = O.detect_zc_peaks(d["corr_mag"], st["above_threshold"], st["metric_valid"],
                                           N, int(d["hysteresis"]))
        assert np.array_equal(ev, d["events"]) and np.array_equal(vals, d["peak_values"])
        assert np.array_equal(mask, d["gate_mask"])
    elif kind == "plateau":
        la = None if int(d["lookahead"]) < 0 else int(d["lookahead"])
        if int(d["error"]):
            with pytest.raises(ValueError):
                O.plateau_end(d["M"], int(d["cp"]), la, int(d["smooth_win"]))
        else:
            idx, _, _ = O.plateau_end(d["M"], int(d["cp"]), la, int(d["smooth_win"]))
            assert idx == int(d["index"])
    elif kind == "minn_peak":
        b = None if int(d["bounds"][0]) < 0 else (int(d["bounds"][0]), int(d["bounds"][1]))
        if int(d["error"]):
            with pytest.raises(ValueError):
                O.minn_peak(d["M"], int(d["smooth_win"]), float(d["thr"]), b)
        else:
            pk, gate, Ms = O.minn_peak(d["M"], int(d["smooth_win"]), float(d["thr"]), b)
            assert pk == int(d["peak"])
            assert np.array_equal(gate, d["gate"]) and np.array_equal(Ms, d["Ms"])   # literal recursion
    elif kind == "trailing":
        assert np.array_equal(O.trailing_average(d["x"], 16), d["y16"])
        assert np.array_equal(O.trailing_average(d["x"], 1), d["y1"])
        assert np.array_equal(O.trailing_average(d["x3"], 3), d["y3"])
    elif kind == "comb_detect":
        mask, span = O.sc_gate(d["M_sc"])
        assert np.array_equal(mask, d["gate"]) and span == tuple(int(v) for v in d["span"])
        assert O.comb_minn_peak(d["M_minn"], int(d["smooth_win"]), mask) == int(d["peak"])
    elif kind == "streaming_peak":
        for j in range(4):
            r = O.streaming_peak(d["metric"], d[f"mask{j}"])
            assert (-1 if r is None else r) == int(d[f"peak{j}"])
    elif kind == "synth":
        pass        # input builders of the synthesis: pinned in tests/test_host_logic.py
    else:
        pytest.fail(kind)


def _csv_rows(name):
    lines = open(os.path.join(GOLDEN, name)).read().splitlines()
    rows = [ln for ln in lines if ln and not ln.startswith("#")]
    return rows[0], rows[1:]


_NEG_ZERO = re.compile(r"-(0\.0+)(?=,|$)")


def unsign_zero(row: str) -> str:
    """'-0.00' -> '0.00': the sign of a ~1e-17 rounding residue is not part of the value
    (the reference's recursive sums and a prefix-sum restatement leave residues of either
    sign where the true P is exactly 0)."""
    return _NEG_ZERO.sub(r"\1", row)


def _fmt_rows(P, R, M, cols, idx):
    out = []
    for n in idx:
        p = P[n]
        if cols[-1] == "R":
            out.append("%d,%.8f,%.2f,%.2f,%.2f,%.2f" % (n, M[n], p.real, p.imag, abs(p) ** 2, R[n]))
        else:
            out.append("%d,%.8f,%.2f,%.2f,%.2f,%.8f" % (n, M[n], p.real, p.imag, abs(p) ** 2, np.angle(p)))
    return out


@pytest.mark.parametrize("csv,case", [("detector_test_vector.csv", "aa_clean_L512"),
                                      ("detector_cfo_test_vector.csv", "aa_cfo_L512")])
def test_oracle_reproduces_reference_csv(csv, case):
    """docs/detector*_test_vector.csv reproduced string-for-string, up to the
    sign of printed zeros."""
    header, rows = _csv_rows(csv)
    cols = header.split(",")
    d = _load(os.path.join(GOLDEN, case + ".npz"))
    P, R, M, _ = O.aa_metric(d["x"], 512)
    idx = [int(r.split(",")[0]) for r in rows]
    assert [unsign_zero(r) for r in _fmt_rows(P, R, M, cols, idx)] == [unsign_zero(r) for r in rows]


def test_preamble_vector_matches_golden_input():
    """docs/preamble_test_vector.csv holds the [A][A] preamble that sits at 500..1523 of the
    detector-vector input; its int12 column is round(x*1024)."""
    d = _load(os.path.join(GOLDEN, "aa_clean_L512.npz"))
    tab = np.genfromtxt(os.path.join(GOLDEN, "preamble_test_vector.csv"), delimiter=",", skip_header=1)
    pre = d["x"][0, 500:1524]
    assert np.max(np.abs(tab[:, 1] - pre.real)) < 1e-9 and np.max(np.abs(tab[:, 2] - pre.imag)) < 1e-9
    assert np.array_equal(tab[:, 3], np.round(pre.real * 1024)) and np.array_equal(tab[:, 4], np.round(pre.imag * 1024))


# ---------------------------------------------------------------------------------------
# closed-form gate/peak formulation (what win_kernel/aa_events implements) vs the loop FSM
# ---------------------------------------------------------------------------------------
def events_closed_form(P, M, valid, L, thr, hyst, fs):
    T = len(M)
    Hp = max(hyst, 1)
    above = valid & (M >= thr)
    pos = np.where(above, np.arange(T), -1)
    prev_incl = np.maximum.accumulate(pos) if T else pos
    prev_excl = np.concatenate([[-1], prev_incl[:-1]]) if T else pos
    n = np.arange(T)
    close = valid & (prev_incl >= 0) & (n - prev_incl == Hp)
    opn = above & ((prev_excl < 0) | (n - 1 - prev_excl >= Hp))
    opens, closes = np.flatnonzero(opn), np.flatnonzero(close)
    pm = np.abs(P) ** 2
    ints, reals = [], []
    for k, o in enumerate(opens):
        c = closes[k] if k < len(closes) else None
        hi = T - 1 if c is None else c
        pk = o + int(np.argmax(pm[o:hi + 1]))
        ints.append((pk, o, T if c is None else c, pk - 2 * L + 1))
        reals.append((P[pk].real, P[pk].imag, M[pk], np.angle(P[pk]) * fs / (2 * np.pi * L)))
    return np.array(ints, np.int64).reshape(-1, 4), np.array(reals).reshape(-1, 4)


@pytest.mark.parametrize("seed", range(40))
def test_closed_form_events_equal_loop_fsm(seed):
    rng = np.random.default_rng(seed)
    T = int(rng.integers(1, 3000))
    L = int(rng.integers(1, 300))
    hyst = int(rng.choice([0, 1, 2, 3, 7, 128]))
    thr = float(rng.uniform(0.05, 0.9))
    # bursty metric so gates open/close many times; |P|² with deliberate ties
    M = np.clip(rng.standard_normal(T).cumsum() * 0.05 + 0.3, 0, 1)
    P = (rng.integers(0, 5, T) + 1j * rng.integers(0, 3, T)).astype(np.complex128)
    valid = np.arange(T) >= L
    ref_i, ref_r = O.aa_events(P, M, valid, L, thr, hyst, 15.36e6)
    cf_i, cf_r = events_closed_form(P, M, valid, L, thr, hyst, 15.36e6)
    assert np.array_equal(ref_i, cf_i)
    assert np.allclose(ref_r, cf_r)


@pytest.mark.parametrize("case", ["aa_clean_L512", "aa_cfo_L512", "aa_grid_len1024_cir1_snr0_fs0.5",
                                  "aa_grid_len256_cir1_snr0_fs1.0", "aa_edge_T15_L8_a2", "aa_edge_T33_L2_a2",
                                  "aa_edge_T5_L8_a1", "aa_int12_L128"])
def test_literal_loop_form_matches_reference_golden(case):
    """The literal per-sample restatement (bench.py's literal-loop CPU baseline) reproduces the
    reference's own outputs: same recursion, so ~ulp agreement (bit-exact on int12 inputs)."""
    d = _load(os.path.join(GOLDEN, case + ".npz"))
    L = int(d["L"])
    P, R, M, valid, ei, er = O.aa_detect_loop(d["x"], L, float(d["threshold"]), int(d["hysteresis"]),
                                              float(d["sample_rate"]))
    scale = max(1.0, float(np.max(np.abs(d["R"]))))
    assert np.max(np.abs(P - d["P"]), initial=0) <= 1e-12 * scale
    assert np.max(np.abs(R - d["R"]), initial=0) <= 1e-12 * scale
    assert np.max(np.abs(M - d["M"]), initial=0) <= 1e-12
    assert np.array_equal(valid, d["valid"])
    assert np.array_equal(ei, d["ev_int"].reshape(-1, 4))
    assert np.allclose(er, d["ev_real"].reshape(-1, 4), rtol=1e-12, atol=1e-9)
    if case == "aa_int12_L128":
        assert np.array_equal(P, d["P"]) and np.array_equal(R, d["R"])
