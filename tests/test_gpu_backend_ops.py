"""GPU parity of the receiver back-end helpers one by one, under the reference's names
(core.py:123-138, 171-176, 339-370, 443-469; sync_aa.py:263-291), against goldens the reference
itself produced (tests/golden/bops_*.npz, make_golden.gen_backend_ops), through the C ABI.

Tolerances (written here):
  ls_channel_estimate / equalize: bit-identical (numpy's complex division restated exactly);
  quantize_adc: bit-identical in both precisions (fp32 for complex64 + Python-float full scale);
  apply_cfo: 4e-16 x max|x| (the tone's sin/cos: device libm vs numpy, ~1 ulp);
  ofdm_fft_used: 1e-12 x max|X| (radix-2 FFT vs pocketfft summation order);
  remove_common_phase / align_complex_gain / evm_rms_db: 1e-12 relative (reduction order);
  estimate_timing_offset_from_phase_slope: 1e-9 relative (atan2 ulps through the fit).
The rebinding of sc.run_simulation's chain (sc.py:274-311) helper by helper equals the fused
ofs_rx_backend kernel and the reference's chain goldens.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import core, sync_aa  # noqa: E402

CASES = ["bops_cir1_2br", "bops_awgn_1br"]


def G(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def close(a, b, tol):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    scale = max(float(np.max(np.abs(b))) if b.size else 0.0, 1e-300)
    err = float(np.max(np.abs(a - b))) / scale if b.size else 0.0
    assert err <= tol, err
    return err


@pytest.mark.parametrize("name", CASES)
def test_apply_cfo_vs_reference(name):
    d = G(name)
    out = core.apply_cfo(d["rx"], float(d["cfo"]), float(d["fs"]))
    assert isinstance(out, np.ndarray) and out.dtype == np.complex128 and out.shape == d["rx_cfo"].shape
    close(out, d["rx_cfo"], 4e-16)
    close(core.apply_cfo(np.atleast_2d(d["rx"])[0], -float(d["cfo"]) / 3, float(d["fs"])), d["rx1_cfo"], 4e-16)
    with pytest.raises(ValueError):
        core.apply_cfo(np.zeros((1, 2, 3), complex), 1.0, 2.0)


@pytest.mark.parametrize("name", CASES)
def test_ofdm_fft_used_vs_reference(name):
    d = G(name)
    for x, y in ((d["sym_p"], d["y_p"]), (d["sym_d"], d["y_d"]), (d["sym_p"][:2048 - 300], d["y_short"])):
        out = core.ofdm_fft_used(x)
        assert out.dtype == np.complex128 and out.shape == (1200,)
        close(out, y, 1e-12)


def test_ofdm_fft_used_truncates_like_numpy():
    d = G("bops_cir1_2br")
    # y_long = ofdm_fft_used(eff[ps : ps + N + 200]): numpy's fft(x, n=N) keeps the first N samples
    x = np.concatenate([d["sym_p"], np.ones(200, complex)])
    np.testing.assert_array_equal(core.ofdm_fft_used(x), core.ofdm_fft_used(d["sym_p"]))


@pytest.mark.parametrize("name", CASES)
def test_ls_and_equalize_bit_identical(name):
    d = G(name)
    h = core.ls_channel_estimate(d["y_p"], d["pil_used"])
    np.testing.assert_array_equal(h, d["h"])
    np.testing.assert_array_equal(core.equalize(d["y_d"], d["h"]), d["xhat"])
    # rows [B, n] with a shared / per-row divisor, device tensors in and out
    Y = torch.from_numpy(np.stack([d["y_p"], d["y_d"]])).cuda()
    H = core.ls_channel_estimate(Y, d["pil_used"])
    assert isinstance(H, torch.Tensor) and H.is_cuda
    np.testing.assert_array_equal(H[0].cpu().numpy(), d["h"])
    E = core.equalize(Y, torch.from_numpy(np.stack([d["h"], d["h"]])).cuda())
    np.testing.assert_array_equal(E[1].cpu().numpy(), d["xhat"])


@pytest.mark.parametrize("name", CASES)
def test_common_phase_gain_evm_vs_reference(name):
    d = G(name)
    x, cpe = core.remove_common_phase(d["xhat"])
    assert isinstance(cpe, float) and abs(cpe - float(d["cpe"])) <= 1e-12 * max(1.0, abs(float(d["cpe"])))
    close(x, d["x_cpe"], 1e-12)
    x, cpe = core.remove_common_phase(d["xhat"], d["dat_used"])
    assert abs(cpe - float(d["cpe_ref"])) <= 1e-12 * max(1.0, abs(float(d["cpe_ref"])))
    close(x, d["x_cpe_ref"], 1e-12)
    xa, g = core.align_complex_gain(d["xhat"], d["dat_used"])
    assert isinstance(g, complex) and abs(g - complex(d["gain"])) <= 1e-12 * abs(complex(d["gain"]))
    close(xa, d["xa"], 1e-12)
    evm, db = core.evm_rms_db(d["xa"], d["dat_used"])
    assert abs(evm - float(d["evm"])) <= 1e-12 * float(d["evm"]) and abs(db - float(d["evm_db"])) <= 1e-10


@pytest.mark.parametrize("name", CASES)
def test_phase_slope_vs_reference(name):
    d = G(name)
    slope, sto = core.estimate_timing_offset_from_phase_slope(d["h"])
    assert abs(slope - float(d["slope"])) <= 1e-9 * max(abs(float(d["slope"])), 1e-12)
    assert abs(sto - float(d["sto"])) <= 1e-9 * max(abs(float(d["sto"])), 1e-9)
    assert core.estimate_timing_offset_from_phase_slope(np.zeros(0, complex)) == (0.0, 0.0)
    with pytest.raises(ValueError):                     # numpy would fail to broadcast k against h
        core.estimate_timing_offset_from_phase_slope(d["h"][:100])


@pytest.mark.parametrize("name", CASES)
def test_quantize_adc_bit_identical(name):
    d = G(name)
    x = np.atleast_2d(d["rx_cfo"])[0]
    rms = float(d["rms"])
    q = sync_aa.quantize_adc(x, 4.0 * rms)
    assert q.dtype == np.complex128
    np.testing.assert_array_equal(q, d["q64"])
    np.testing.assert_array_equal(sync_aa.quantize_adc(x, np.float64(2.5 * rms), bits=8), d["q64_np"])
    q32 = sync_aa.quantize_adc(d["x32"], 3.0 * rms)                # float32 arithmetic, complex64 out
    assert q32.dtype == np.complex64
    np.testing.assert_array_equal(q32, d["q32"])
    q32n = sync_aa.quantize_adc(d["x32"], np.float64(3.0 * rms))   # float64 full scale promotes
    assert q32n.dtype == np.complex128
    np.testing.assert_array_equal(q32n, d["q32_np"])


@pytest.mark.parametrize("name", ["backend_cir1_2br", "backend_awgn_1br", "backend_cir2_2br_early"])
def test_run_simulation_chain_rebound_helper_by_helper(name):
    """sc.run_simulation's back-end (sc.py:274-311) with every core helper rebound to the GPU
    drop-ins, as INTEGRATION.md shows: equals the reference's chain goldens and the fused kernel."""
    d = G(name)
    rx, ps, ds = d["x"], int(d["pilot_start"]), int(d["data_start"])
    N, CP, fs = int(d["n_fft"]), int(d["cp"]), float(d["fs"])
    cfo = core.estimate_cfo_from_cp(rx, ps, N, CP, fs)
    rxc = core.apply_cfo(rx, -cfo, fs)
    eff = rxc if rxc.ndim == 1 else np.mean(rxc, axis=0)
    h = core.ls_channel_estimate(core.ofdm_fft_used(eff[ps + CP:ps + CP + N]), d["pilot_used"])
    slope, sto = core.estimate_timing_offset_from_phase_slope(h)
    xhat = core.equalize(core.ofdm_fft_used(eff[ds + CP:ds + CP + N]), h)
    xa, gain = core.align_complex_gain(xhat, d["data_used"])
    evm, evm_db = core.evm_rms_db(xa, d["data_used"])
    assert abs(cfo - float(d["cfo"])) < 1e-9
    close(h, d["h"], 1e-11)
    close(xa, d["xa"], 1e-10)
    assert abs(evm - float(d["evm"])) <= 1e-10 * float(d["evm"])
    assert abs(slope - float(d["slope"])) <= 1e-8 * max(abs(float(d["slope"])), 1e-12)
    fused = core.receiver_backend(rx, ps, ds, d["pilot_used"], d["data_used"])
    close(fused["h"], h, 1e-11)
    assert abs(fused["evm"] - evm) <= 1e-10 * evm


def test_division_broadcasts_like_numpy_and_empty_paths():
    """A [n] numerator against [B, n] divisors broadcasts to [B, n] like numpy's Y / (X + eps);
    remove_common_phase of an empty list returns an ndarray copy and nan; outputs are complex128
    (the helpers compute in fp64 whatever the input precision)."""
    rng = np.random.default_rng(8)
    y = rng.standard_normal(40) + 1j * rng.standard_normal(40)
    d = rng.standard_normal((3, 40)) + 1j * rng.standard_normal((3, 40))
    h = core.ls_channel_estimate(y, d)
    assert h.shape == (3, 40) and h.dtype == np.complex128
    np.testing.assert_array_equal(h, y / (d + 1e-9))
    x, cpe = core.remove_common_phase([])
    assert isinstance(x, np.ndarray) and x.size == 0 and np.isnan(cpe)
    h64 = core.equalize(y.astype(np.complex64), d[0].astype(np.complex64))
    assert h64.dtype == np.complex128
    np.testing.assert_allclose(h64, y.astype(np.complex64).astype(np.complex128) /
                               (d[0].astype(np.complex64).astype(np.complex128) + 1e-9), rtol=1e-15)
