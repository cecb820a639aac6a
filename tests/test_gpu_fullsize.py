"""GPU: BASELINE.json configurations at their full per-GPU sizes, checked through
size-independent properties plus oracle parity on sampled streams.

  cfg2  4096 x 1024 int12 streams: sync_aa L=128 and minn_rtl Q=64 on the integer-exact kernels,
        bit-identical to the general engine (fp64, sequential IIR) on EVERY stream, the oracle on
        a sample (exact integers);
  cfg4  32768 x 4096 c64 (one GPU's shard of 262144), fused combined S&C + Minn, N = 2048:
        oracle on a sample (M 1e-6), combined S&C M <= 1/4 and Minn M >= 0 on every stream;
  cfg5  262144 x 4096 c64 (a quarter of 1M; the full 32 GiB run is bench_configs' job),
        zc_freq fp32 window FFT: oracle on a sample (2e-5 abs), 0 <= metric <= 1 everywhere.
"""
import numpy as np
import pytest

import ofdm_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import _lib, combined_sc_min, minn_rtl, sync_aa, synth, zc_freq  # noqa: E402


def int12_batch(B, T, L, seed):
    return synth.synth_batch(synth.faded_base(L, "cir1", (0, 1)), B, T, seed=seed, dtype=torch.int16,
                             adc_scale=700.0)


def test_cfg2_sync_aa_full_batch_exact(monkeypatch):
    B, T, L = 4096, 1024, 128
    x = int12_batch(B, T, L, 21)
    assert _lib.lib().ofs_aa_plan(_lib.CI16, _lib.FP64, 2, T, L) > 2000
    a = sync_aa.aa_detect_streaming_batched(x, L=L)
    monkeypatch.setenv("OFS_EXACT", "0")
    g = sync_aa.aa_detect_streaming_batched(x, L=L)
    monkeypatch.delenv("OFS_EXACT")
    for k in ("P", "R", "M", "valid", "n_events"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    n = a.n_events.cpu().numpy()
    assert (n >= 1).mean() > 0.9
    m = int(min(n.max(), a.ev_int.shape[1]))
    live = (torch.arange(m, device=a.ev_int.device)[None, :] < a.n_events[:, None])[..., None]   # stored slots
    assert torch.equal(torch.where(live, a.ev_int[:, :m], 0), torch.where(live, g.ev_int[:, :m], 0))
    xi = x.cpu().numpy()
    for b in np.linspace(0, B - 1, 6).astype(int):
        xc = (xi[b, ..., 0] + 1j * xi[b, ..., 1]).astype(np.complex128)
        P, R, M, v = O.aa_metric(xc, L)
        assert np.array_equal(a.P[b].cpu().numpy(), P)


def test_cfg2_minn_rtl_full_batch_exact(monkeypatch):
    B, T, Q = 4096, 1024, 64
    x = int12_batch(B, T, 2 * Q, 22)
    assert _lib.lib().ofs_rtl_plan(_lib.CI16, 2, T, Q) > 2000
    a = minn_rtl.minn_rtl_batched(x, Q, hysteresis=2)
    monkeypatch.setenv("OFS_EXACT", "0")
    g = minn_rtl.minn_rtl_batched(x, Q, hysteresis=2)
    monkeypatch.delenv("OFS_EXACT")
    for k in ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled", "energy_scaled",
              "metric_valid", "above_threshold", "n_events", "open_gate_start"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    xi = x.cpu().numpy()
    b = B // 3
    xc = (xi[b, ..., 0] + 1j * xi[b, ..., 1]).astype(np.complex128)
    s = O.minn_rtl_metric(xc, Q, minn_rtl.SMOOTH_SHIFT, minn_rtl.THRESH_VALUE, minn_rtl.THRESH_FRAC_BITS)
    assert np.array_equal(a.smooth_metric[b].cpu().numpy(), s["smooth_metric"])


def test_cfg4_fused_shard_full_size():
    B, T, N = 32768, 4096, 2048
    x = synth.make_aa_batch(B, T, N // 2, seed=4, device="cuda")
    (Mm, Pm, Rm), (Ms, Ps, Rs) = combined_sc_min.sc_minn_streaming_metrics_batched(x, N)
    assert Ms.shape == (B, T - N + 1)
    assert bool(torch.isfinite(Ms).all()) and bool(torch.isfinite(Mm).all())
    assert float(Ms.max()) <= 0.25 + 1e-6 and float(Mm.min()) >= 0.0       # |P| <= (E1+E2)/2
    xh = x[:: B // 8].cpu().numpy().astype(np.complex128)
    for i, b in enumerate(range(0, B, B // 8)):
        Mo, Po, Ro = O.comb_sc_metric(xh[i], N)
        assert np.max(np.abs(Ms[b].cpu().numpy() - Mo)) < 1e-6
        Mo, Po, Ro = O.minn_metric(xh[i], N)
        mm = Mm[b].cpu().numpy()
        assert np.all(np.abs(mm - Mo) <= 1e-6 * np.maximum(1.0, np.abs(Mo)))


def test_cfg5_quarter_batch():
    B, N = 262144, 4096
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn((B, N), dtype=torch.complex64, device="cuda", generator=g)
    sym = torch.from_numpy(O.pss_symbol(N).astype(np.complex64)).cuda()
    x[::97] += 4.0 * sym                                                 # some windows carry the PSS
    idx, t, e = O.zc_template()
    m = zc_freq.compute_frequency_metric_batched(x, idx, t, e, N=N, cp=0)
    assert m.shape == (B, 1)
    assert float(m.min()) >= 0.0 and float(m.max()) <= 1.0 + 1e-5        # Cauchy-Schwarz
    assert float(m[::97].min()) > 0.5
    for b in list(range(0, B, B // 12)) + [97, 194]:
        mo = O.zc_freq_metric(x[b].cpu().numpy().astype(np.complex128)[None], N, 0, idx, t, e)
        assert abs(float(m[b, 0]) - mo[0]) < 2e-5
