"""GPU parity for the rocFFT leg of the ZC frequency-domain metric (csrc/zc_rocfft.hip,
ofs_zc_freq_metric_fft) and the per-stream first-argmax kernel (ofs_row_argmax), through the
C ABI: against the reference goldens (zc_freq.py:62-99 with N_FFT overridden), the CPU oracle,
numpy's argmax (zc_freq.py:144) and the fused window-FFT kernel of ofs_zc_freq_metric.

Tolerances (written here): complex128 input (rocFFT double + fp64 gather): 1e-9 relative +
1e-11 absolute (pocketfft vs rocFFT summation order); complex64 input (rocFFT single, fp64
gather): every window within fp32 error model 2 of tests/error_models.py (eps of an all-fp32
log2(N)-stage FFT), checked by oracle_zc_freq_check, measured ratio printed.  Argmax indices
exact on fp64.
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

from ofdm_sync_amd import _lib, zc_freq  # noqa: E402


def G(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def rng_c(rng, *shape):
    return rng.standard_normal(shape) + 1j * rng.standard_normal(shape)


@pytest.mark.parametrize("name", ["zcfreq_N2048", "zcfreq_N256"])
def test_rocfft_vs_reference_golden(name):
    d = G(name)
    N, cp = int(d["N"]), int(d["CP"])
    idx, t, e = zc_freq.make_pss_frequency_template()
    x = np.asarray(d["x"])
    x = x[None] if x.ndim == 1 else x                 # (branches, T) -> one stream
    m, pk, pv = zc_freq.compute_frequency_metric_rocfft_batched(torch.from_numpy(x[None].astype(np.complex128)).cuda(),
                                                                idx, t, e, N=N, cp=cp, return_peak=True)
    assert m.dtype == torch.float64 and m.shape == (1,) + d["metric"].shape
    np.testing.assert_allclose(m[0].cpu().numpy(), d["metric"], rtol=1e-9, atol=1e-11)
    assert int(pk[0]) == int(np.argmax(d["metric"]))
    assert float(pv[0]) == pytest.approx(float(np.max(d["metric"])), rel=1e-9)


@pytest.mark.parametrize("N,cp,T,nb", [(256, 64, 400, 1), (256, 64, 420, 2), (128, 0, 200, 3), (64, 16, 80, 1)])
def test_rocfft_fp64_vs_oracle(N, cp, T, nb):
    rng = np.random.default_rng(N * 3 + nb)
    B = 5
    x = rng_c(rng, B, nb, T)
    idx, t, e = O.zc_template()
    if T >= 40 + N:
        x[2, :, 40:40 + N] += 4 * O.pss_symbol(N)
    m, pk, _ = zc_freq.compute_frequency_metric_rocfft_batched(torch.from_numpy(x).cuda(), idx, t, e, N=N, cp=cp,
                                                               return_peak=True)
    mm = m.cpu().numpy()
    for b in range(B):
        mo = O.zc_freq_metric(x[b], N, cp, idx, t, e)
        np.testing.assert_allclose(mm[b], mo, rtol=1e-9, atol=1e-11)
        assert int(pk[b]) == int(np.argmax(mm[b]))


@pytest.mark.parametrize("B,nb,cp,T", [(1000, 1, 0, 4096), (64, 2, 512, 4610)])
def test_rocfft_fp32_cfg5_shape_vs_oracle_and_fused(B, nb, cp, T):
    """cfg5 shape (N = 4096, complex64): rocFFT leg vs oracle, and vs the fused window-FFT kernel."""
    N = 4096
    rng = np.random.default_rng(B + nb)
    x = rng_c(rng, B, nb, T)
    sym = O.pss_symbol(N)
    for b in range(0, B, 4):
        x[b, :, cp:cp + N] += rng.uniform(0.5, 8.0) * sym
    x = x.astype(np.complex64)
    idx, t, e = O.zc_template()
    xd = torch.from_numpy(x).cuda()
    m = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp)
    assert m.dtype == torch.float32
    mf = zc_freq.compute_frequency_metric_batched(xd, idx, t, e, N=N, cp=cp)
    mm = m.cpu().numpy()
    for v, eps, name in ((mm, EM.rocfft_eps(N), "rocFFT"), (mf.cpu().numpy(), EM.zc_win_eps(N), "fused")):
        st = oracle_c.zc_freq_check(x, N, cp, idx, t, e, v, eps, 6.0)
        print(f"{name} B={B} nb={nb}: max |dm| {st[:, 0].max():.3g}, max |dm|/bound {st[:, 1].max():.3g}")
        assert st[:, 1].max() <= 1.0
    assert mm.max() > 0.5


def test_rocfft_too_short_and_bad_input():
    idx, t, e = O.zc_template()
    with pytest.raises(ValueError):
        zc_freq.compute_frequency_metric_rocfft_batched(torch.ones((2, 79), dtype=torch.complex64).cuda(),
                                                        idx, t, e, N=64, cp=16)
    m = zc_freq.compute_frequency_metric_rocfft_batched(torch.ones((2, 80), dtype=torch.complex64).cuda(),
                                                        idx, t, e, N=64, cp=16)
    assert m.shape == (2, 1)
    with pytest.raises(ValueError):
        zc_freq.compute_frequency_metric_rocfft_batched(torch.ones((2, 80, 2), dtype=torch.int16).cuda(),
                                                        idx, t, e, N=64, cp=16)


@pytest.mark.parametrize("n", [1000, 33, 32, 7])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_row_argmax_numpy_semantics(dtype, n):
    """Wave-per-row kernel (n > 32) and thread-per-row kernel (n <= 32): numpy's first argmax."""
    rng = np.random.default_rng(7)
    v = rng.integers(0, 5, size=(300, n)).astype(np.float64)     # many ties: first index must win
    v[3, :] = -np.inf
    v[4, n // 2] = np.nan
    v[4, n - 1] = np.nan
    v[8, 0] = np.nan
    v[5, n - 1] = 100.0
    v[6, 0] = 100.0
    v[7, :] = 1.0
    idx, val = zc_freq.peak_index_batched(torch.from_numpy(v).to(dtype).cuda())
    ref = np.argmax(v, axis=1)
    assert np.array_equal(idx.cpu().numpy(), ref)
    vv = val.cpu().numpy()
    for b in range(v.shape[0]):
        if not np.isnan(v[b, ref[b]]):
            assert vv[b] == v[b, ref[b]]
    idx1, _ = zc_freq.peak_index_batched(torch.tensor([[2.0]], dtype=dtype).cuda())
    assert int(idx1[0]) == 0


@pytest.mark.parametrize("prec,N,cp,T,nb", [("c128", 256, 32, 700, 2), ("c64", 4096, 0, 4096, 1), ("c64", 2048, 0, 2300, 2)])
def test_pruned_store_callback_equals_dense(prec, N, cp, T, nb):
    """The pruned plan (rocFFT store callback keeping the 62 template bins) gives the dense plan's
    metric: same transform, only the write of the unused bins is skipped."""
    rng = np.random.default_rng(N + T)
    B = 9
    x = rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))
    xd = torch.from_numpy(x.astype(np.complex128 if prec == "c128" else np.complex64)).cuda()
    idx, t, e = zc_freq.make_pss_frequency_template()
    a, pa, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True, pruned=True,
                                                               layout="offsets")
    b, pb, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True, pruned=False,
                                                               layout="offsets")
    tol = 1e-12 if prec == "c128" else 1e-5
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=tol, atol=tol * 1e-3)
    if prec == "c128":
        ref = np.stack([O.zc_freq_metric(x[k], N, cp, idx, t, e) for k in range(B)])
        np.testing.assert_allclose(a.cpu().numpy(), ref, rtol=1e-9, atol=1e-7)
    else:
        st = oracle_c.zc_freq_check(x.astype(np.complex64), N, cp, idx, t, e, a.cpu().numpy(), EM.rocfft_eps(N), 6.0)
        print(f"pruned c64 N={N}: max |dm|/bound {st[:, 1].max():.3g}")
        assert st[:, 1].max() <= 1.0


@pytest.mark.parametrize("prec,nb,chunk,pruned", [("c128", 1, 7, False), ("c128", 2, 6, False), ("c64", 3, 9, False),
                                                  ("c64", 2, 4, True), ("c64", 1, 64, False)])
def test_rocfft_chunked_equals_one_execution(prec, nb, chunk, pruned):
    """Chunked plans (ofs_zc_fft_plan_create3: rocFFT executions over `chunk` windows into one
    reused spectrum buffer, chunk not dividing the batch -> a tail plan) give the one-execution
    result, several offsets per stream; fp64 also against the oracle."""
    N, cp, T, B = 256, 32, 300, 23
    rng = np.random.default_rng(chunk * 7 + nb)
    x = rng_c(rng, B, nb, T)
    x[3, :, cp + 5:cp + 5 + N] += 3 * O.pss_symbol(N)
    x = x.astype(np.complex128 if prec == "c128" else np.complex64)
    idx, t, e = O.zc_template()
    xd = torch.from_numpy(x).cuda()
    m0, pk0, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True,
                                                                 pruned=pruned, chunk=0, layout="offsets")
    m1, pk1, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True,
                                                                 pruned=pruned, chunk=chunk, layout="offsets")
    a0, a1 = m0.cpu().numpy(), m1.cpu().numpy()
    tol = dict(rtol=1e-9, atol=1e-11)
    if prec == "c128":
        np.testing.assert_allclose(a1, a0, **tol)
    else:                                        # the same rocFFT transform per window: model 2 both
        for v in (a0, a1):
            assert oracle_c.zc_freq_check(x, N, cp, idx, t, e, v, EM.rocfft_eps(N), 6.0)[:, 1].max() <= 1.0
    if prec == "c128":
        assert torch.equal(pk0, pk1)
        for b in (0, 3, B - 1):
            np.testing.assert_allclose(a1[b], O.zc_freq_metric(x[b], N, cp, idx, t, e), **tol)
    assert int(pk1[3]) == 5


def test_rocfft_chunk_must_split_branches():
    idx, t, e = O.zc_template()
    with pytest.raises(ValueError):
        zc_freq.compute_frequency_metric_rocfft_batched(torch.ones((4, 2, 80), dtype=torch.complex64).cuda(),
                                                        idx, t, e, N=64, cp=16, chunk=3)


@pytest.mark.parametrize("pruned", [False, True])
@pytest.mark.parametrize("prec,N,cp,T,nb,B,rpe", [("c128", 2048, 512, 4242, 2, 5, 0), ("c128", 2048, 512, 4242, 2, 5, 4),
                                                  ("c64", 2048, 512, 4242, 2, 64, 0), ("c128", 256, 32, 700, 3, 7, 6),
                                                  ("c64", 128, 0, 1000, 1, 33, 5)])
def test_rocfft_rows_layout_equals_offsets(prec, N, cp, T, nb, B, rpe, pruned):
    """The rows plan (ofs_zc_fft_plan_create_rows: every offset of a row group in ONE rocFFT execution,
    windows one sample apart; dense spectrum rows by default, or the store callback keeping the template
    bins of the windows inside one row with pruned=True) gives the per-offset plan's metric and argmax on
    the reference's own sliding shape (T = 4242, 2 branches, N = 2048, cp = 512: 1683 offsets), with row
    groups that leave a tail; fp64 also vs the oracle, complex64 within error model 2 on every window."""
    rng = np.random.default_rng(N + T + B)
    x = rng_c(rng, B, nb, T)
    sym = O.pss_symbol(N)
    for b in range(0, B, 3):
        s0 = int(rng.integers(0, T - N - cp))
        x[b, :, s0 + cp:s0 + cp + N] += 3 * sym
    x = x.astype(np.complex128 if prec == "c128" else np.complex64)
    idx, t, e = O.zc_template()
    xd = torch.from_numpy(x).cuda()
    r, pr, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True,
                                                               layout="rows", rows_per_execution=rpe, pruned=pruned)
    o, po, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True,
                                                               layout="offsets", pruned=True)
    a, b_ = r.cpu().numpy(), o.cpu().numpy()
    assert a.shape == (B, T - N - cp + 1)
    if prec == "c128":
        np.testing.assert_allclose(a, b_, rtol=1e-12, atol=1e-14)
        assert torch.equal(pr, po)
        for k in (0, B - 1):
            np.testing.assert_allclose(a[k], O.zc_freq_metric(x[k], N, cp, idx, t, e), rtol=1e-9, atol=1e-11)
    else:
        st = oracle_c.zc_freq_check(x, N, cp, idx, t, e, a, EM.rocfft_eps(N), 6.0)
        print(f"rows c64 N={N} pruned={pruned}: max |dm|/bound {st[:, 1].max():.3g}")
        assert st[:, 1].max() <= 1.0
        np.testing.assert_allclose(a, b_, rtol=1e-5, atol=1e-8)


def test_rocfft_rows_execution_beyond_grid_y_limit():
    """One rows-plan execution over more than 65535 streams: zc_gather_rows_kernel strides its streams
    over gridDim.y (<= 65535), so the launch still covers every stream (advisor, round 5); the metric
    equals the per-offset plan's (fp32, different rocFFT plans: within 1e-5), the peaks its own argmax."""
    N, cp, T, B = 64, 0, 66, 66000
    rng = np.random.default_rng(5)
    x = rng_c(rng, B, 1, T).astype(np.complex64)
    idx, t, e = O.zc_template()
    xd = torch.from_numpy(x).cuda()
    r, pr, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True,
                                                               layout="rows", rows_per_execution=B)
    o, po, _ = zc_freq.compute_frequency_metric_rocfft_batched(xd, idx, t, e, N=N, cp=cp, return_peak=True,
                                                               layout="offsets")
    assert r.shape == (B, T - N - cp + 1)
    np.testing.assert_allclose(r.cpu().numpy(), o.cpu().numpy(), rtol=1e-5, atol=1e-8)
    rn = r.cpu().numpy()
    assert np.array_equal(pr.cpu().numpy(), np.argmax(rn, axis=1))     # every stream's row was written
