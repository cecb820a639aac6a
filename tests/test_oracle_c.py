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
