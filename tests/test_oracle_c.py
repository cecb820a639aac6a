"""CPU: the C oracle (literal streaming restatement, used as the timed CPU baseline) against
the reference's golden vectors and the NumPy oracle."""
import glob
import os

import numpy as np
import pytest

import oracle_c
import ofdm_oracle as O
from conftest import GOLDEN

AA = [p for p in sorted(glob.glob(os.path.join(GOLDEN, "aa_*.npz")))]


@pytest.mark.parametrize("path", AA, ids=lambda p: os.path.basename(p)[:-4])
def test_c_oracle_matches_reference_golden(path):
    d = np.load(path)
    x = d["x"][None]
    r = oracle_c.aa_detect(x, int(d["L"]), float(d["threshold"]), int(d["hysteresis"]),
                           float(d["sample_rate"]), max_events=8)
    scale = max(1.0, float(np.abs(d["P"]).max(initial=0)))
    assert np.max(np.abs(r["P"][0] - d["P"]), initial=0) <= 1e-13 * scale
    assert np.max(np.abs(r["M"][0] - d["M"]), initial=0) <= 1e-13
    n = int(r["n_events"][0])
    assert n == len(d["ev_int"])
    assert np.array_equal(r["ev_int"][0, :n], d["ev_int"])
    assert np.allclose(r["ev_real"][0, :n], d["ev_real"], rtol=1e-12, atol=1e-9)


def test_c_oracle_batched_c64_threads():
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((37, 2, 900)) + 1j * rng.standard_normal((37, 2, 900))).astype(np.complex64)
    r1 = oracle_c.aa_detect(x, 64, 0.05, 4, nthreads=1)
    r4 = oracle_c.aa_detect(x, 64, 0.05, 4, nthreads=4)
    assert np.array_equal(r1["M"], r4["M"]) and np.array_equal(r1["ev_int"], r4["ev_int"])
    for b in (0, 17, 36):
        P, R, M, v = O.aa_metric(x[b].astype(np.complex128), 64)
        assert np.max(np.abs(r1["M"][b] - M)) < 1e-12


RTL = [p for p in sorted(glob.glob(os.path.join(GOLDEN, "rtl_*.npz")))]


@pytest.mark.parametrize("path", RTL, ids=lambda p: os.path.basename(p)[:-4])
def test_c_minn_rtl_matches_reference_golden(path):
    """The C restatement of minn_rtl's streaming pipeline + detect_minn_rtl (float smoothing)
    reproduces the reference's arrays bit for bit and its events exactly."""
    d = np.load(path)
    r = oracle_c.minn_rtl(d["x"][None], int(d["Q"]), int(d["smooth_shift"]), int(d["threshold_value"]),
                          int(d["threshold_frac_bits"]), int(d["hysteresis"]), int(d["timing_offset"]))
    for k in ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled", "energy_scaled"):
        assert np.array_equal(r[k][0], d[k]), k
    assert np.array_equal(r["metric_valid"][0].astype(bool), d["metric_valid"])
    assert np.array_equal(r["above_threshold"][0].astype(bool), d["above_threshold"])
    n = int(r["n_events"][0])
    assert np.array_equal(r["events"][0, :n], d["events"].reshape(-1, 4))


# ----------------------------------------------------------------------------------------------
# The full-batch checkers that decide cfg4 / cfg5 (tests/test_gpu_fullsize.py), pinned on their
# own: fed the reference's fp64 outputs they must agree to fp64 resolution, and a perturbation of
# 2x the stated error-model bound on one output must come out as a bound ratio of ~2 (> 1), so the
# bounds cannot be vacuous (an inflated S, R or rho would show up as a ratio well below 2).
# ----------------------------------------------------------------------------------------------
import error_models as EM  # noqa: E402


def _comb_goldens():
    c = np.load(os.path.join(GOLDEN, "comb_sc_N2048_cir1_2br.npz"))
    m = np.load(os.path.join(GOLDEN, "comb_minn_N2048_cir1_2br.npz"))
    assert np.array_equal(c["x"], m["x"]) and int(c["N"]) == int(m["N"])
    return c["x"], int(c["N"]), c, m


def test_sc_minn_checker_pinned_to_reference_golden():
    """oracle_sc_minn_check against combined_sc_min.py:60-164's own fp64 outputs (golden
    comb_{sc,minn}_N2048_cir1_2br, 2 branches): |dM| <= 1e-12 for both metrics and every P/R/M
    ratio to the fp32 bounds <= 1e-5 (i.e. agreement far below fp32 resolution)."""
    x, N, c, m = _comb_goldens()
    kP, kR, kM = EM.win_fast_k(4, x.shape[0])
    st = oracle_c.sc_minn_check(x[None], N, c["M"][None], c["P"][None], c["R"][None], m["M"][None],
                                m["P"][None], m["R"][None], kP, kR, kM)[0]
    s = dict(zip(oracle_c.SC_MINN_STATS, st))
    print("checker vs reference fp64:", {k: float(f"{v:.3g}") for k, v in s.items()})
    assert s["comb_max_dM"] <= 1e-12 and s["minn_max_dM_rel1"] <= 1e-12
    for k in ("comb_dM_over_bound", "comb_dP_over_bound", "comb_dR_over_bound", "minn_dM_over_bound",
              "minn_dP_over_bound", "minn_dR_over_bound"):
        assert s[k] <= 1e-5, k


@pytest.mark.parametrize("which", ["comb_M", "comb_P", "comb_R", "minn_M", "minn_P", "minn_R"])
def test_sc_minn_checker_bound_can_fail(which):
    """The reference outputs rounded to fp32 (a valid engine: ratio well below 1), then one output
    perturbed by 2x its error-model bound (tests/error_models.py model 1, evaluated in numpy): the
    checker must report a ratio in (1.5, 2.5) for that quantity."""
    x, N, c, m = _comb_goldens()
    kP, kR, kM = EM.win_fast_k(4, x.shape[0])
    out = {k: {q: np.array(g[q], dtype=np.complex64 if q == "P" else np.float32) for q in "MPR"}
           for k, g in (("comb", c), ("minn", m))}
    base = oracle_c.sc_minn_check(x[None], N, *(out["comb"][q][None] for q in "MPR"),
                                  *(out["minn"][q][None] for q in "MPR"), kP, kR, kM)[0]
    assert max(base[1], base[2], base[3], base[5], base[6], base[7]) < 1.0
    kind, q = which.split("_")
    g = c if kind == "comb" else m
    bM, bP, bR = EM.window_model(kind, x, N, g["P"], g["R"], g["M"], E=4)
    d = int(np.argmax(g["M"]))                        # the preamble peak: every bound is non-trivial
    if q == "M":
        out[kind]["M"][d] = np.float32(g["M"][d] + 2.0 * bM[d])
    elif q == "P":
        out[kind]["P"][d] = np.complex64(g["P"][d] + 2.0 * bP[d])
    else:
        out[kind]["R"][d] = np.float32(g["R"][d] + 2.0 * bR[d])
    st = oracle_c.sc_minn_check(x[None], N, *(out["comb"][q_][None] for q_ in "MPR"),
                                *(out["minn"][q_][None] for q_ in "MPR"), kP, kR, kM)[0]
    col = {("comb", "M"): 1, ("comb", "P"): 2, ("comb", "R"): 3,
           ("minn", "M"): 5, ("minn", "P"): 6, ("minn", "R"): 7}[(kind, q)]
    print(which, "ratio", st[col])
    assert 1.5 < st[col] < 2.5, (which, st[col])


def test_zc_freq_checker_pinned_to_reference_golden():
    """oracle_zc_freq_check against zc_freq.py:62-99's own fp64 metric (goldens zcfreq_N2048 /
    zcfreq_N256, 2 branches, every offset): |dm| <= 1e-12 and the ratio to the fp32 model-2
    bound <= 1e-4."""
    for name in ("zcfreq_N2048", "zcfreq_N256"):
        d = np.load(os.path.join(GOLDEN, name + ".npz"))
        N, cp = int(d["N"]), int(d["CP"])
        st = oracle_c.zc_freq_check(d["x"][None], N, cp, d["bins"], d["template"], float(d["template_energy"]),
                                    d["metric"][None].astype(np.float64), EM.zc_win_eps(N), 6.0)[0]
        print(name, "max |dm|", st[0], "ratio", st[1])
        assert st[0] <= 1e-12 and st[1] <= 1e-4, name


def _zc_bound_numpy(x, N, cp, idx, t, e, off, eps, kM=6.0):
    """Model 2 at one offset, evaluated in numpy (np.fft, as the reference): the bound of |dm|."""
    nb = x.shape[0]
    b = np.concatenate([np.fft.fft(x[br, off + cp:off + cp + N])[np.asarray(idx) % N] for br in range(nb)])
    tt = np.tile(np.asarray(t), nb)
    D = float(np.sum(np.abs(b) ** 2))
    mm = abs(np.vdot(tt, b)) ** 2 / max(e * D, 1e-12)
    W2 = float(np.sum(np.abs(x[:, off + cp:off + cp + N]) ** 2))
    rho = eps * np.sqrt(N) * np.sqrt(W2) / np.sqrt(D)
    return 2.0 * (np.sqrt(nb * mm) + mm) * rho + (nb + 1) * rho ** 2 + kM * 2.0 ** -24 * mm, mm


@pytest.mark.parametrize("name", ["zcfreq_N2048", "zcfreq_N256"])
def test_zc_freq_checker_bound_can_fail(name):
    """One metric value perturbed by 2x its model-2 bound (evaluated in numpy): the checker's
    ratio must be ~2; the unperturbed fp32-rounded reference metric stays below 1."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    N, cp, e = int(d["N"]), int(d["CP"]), float(d["template_energy"])
    x, eps = d["x"], EM.zc_win_eps(N)
    m32 = d["metric"].astype(np.float32)
    base = oracle_c.zc_freq_check(x[None], N, cp, d["bins"], d["template"], e, m32[None], eps, 6.0)[0]
    assert base[1] < 1.0
    off = int(np.argmax(d["metric"]))
    bound, mm = _zc_bound_numpy(x, N, cp, d["bins"], d["template"], e, off, eps)
    assert abs(mm - d["metric"][off]) <= 1e-12
    mp = d["metric"].copy()
    mp[off] += 2.0 * bound
    st = oracle_c.zc_freq_check(x[None], N, cp, d["bins"], d["template"], e, mp[None], eps, 6.0)[0]
    print(name, "perturbed ratio", st[1])
    assert 1.5 < st[1] < 2.5
