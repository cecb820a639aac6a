"""GPU: BASELINE.json configurations at their full per-GPU sizes, checked through
size-independent properties plus oracle parity on sampled streams.

  cfg2  4096 x 1024 int12 streams: sync_aa L=128 and minn_rtl Q=64 on the integer-exact kernels,
        bit-identical to the general engine (fp64, sequential IIR) AND to the C oracle (the
        reference's streaming loops restated statement for statement) on EVERY stream: every
        array bit for bit, every event;
  cfg3  detect-only (events without P/R/M) on the full 65536 x 1024 batch: every stream's events
        against the C oracle under oracle/parity.py's stated near-tie criterion;
  cfg4  32768 x 4096 c64 (one GPU's shard of 262144), fused combined S&C + Minn, N = 2048:
        EVERY stream and output against the C oracle's fp64 values (oracle_sc_minn_check): M, P,
        R within the fp32 error model of tests/error_models.py (model 1), combined S&C M within
        the north-star 1e-6 absolute, Minn M within 1e-6·max(1, M);
  cfg5  the full 1M x 4096 c64 batch (32 GiB), zc_freq fp32 window FFT: EVERY sequence against
        the C oracle's fp64 FFT (oracle_zc_freq_check) within error model 2.
Each test prints the measured maximum error and its ratio to the bound.
"""
import numpy as np
import pytest

import error_models as EM
import ofdm_oracle as O
import oracle_c

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import _lib, combined_sc_min, minn_rtl, sync_aa, synth, zc_freq  # noqa: E402


def int12_batch(B, T, L, seed):
    return synth.synth_batch(synth.faded_base(L, "cir1", (0, 1)), B, T, seed=seed, dtype=torch.int16,
                             adc_scale=700.0)


def test_cfg2_sync_aa_full_batch_exact(variant):
    B, T, L = 4096, 1024, 128
    x = int12_batch(B, T, L, 21)
    assert _lib.lib().ofs_aa_plan(_lib.CI16, _lib.FP64, 2, T, L) > 2000
    a = sync_aa.aa_detect_streaming_batched(x, L=L)
    variant("EXACT", 0)
    g = sync_aa.aa_detect_streaming_batched(x, L=L)
    variant("EXACT", None)
    for k in ("P", "R", "M", "valid", "n_events"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    n = a.n_events.cpu().numpy()
    assert (n >= 1).mean() > 0.9
    m = int(min(n.max(), a.ev_int.shape[1]))
    live = (torch.arange(m, device=a.ev_int.device)[None, :] < a.n_events[:, None])[..., None]   # stored slots
    assert torch.equal(torch.where(live, a.ev_int[:, :m], 0), torch.where(live, g.ev_int[:, :m], 0))
    xi = x.cpu().numpy()
    xc = (xi[..., 0] + 1j * xi[..., 1]).astype(np.complex128)                # [B, 2, T]
    o = oracle_c.aa_detect(xc, L, max_events=int(a.ev_int.shape[1]), nthreads=16)
    assert np.array_equal(a.P.cpu().numpy(), o["P"])                          # exact integer sums
    # R: the engine sums re²+im² (exact integers); the reference (and its C restatement) squares
    # np.abs(x) = hypot(re, im), which is off by an ulp for some samples (sync_aa.py:475-477)
    np.testing.assert_allclose(a.R.cpu().numpy(), o["R"], rtol=1e-14, atol=0)
    np.testing.assert_allclose(a.M.cpu().numpy(), o["M"], rtol=1e-14, atol=0)   # hypot² vs re²+im²
    assert np.array_equal(n, o["n_events"])
    ei = a.ev_int.cpu().numpy()
    er = a.ev_real.cpu().numpy()
    for b in range(B):
        k = min(int(n[b]), ei.shape[1])
        assert np.array_equal(ei[b, :k], o["ev_int"][b, :k])
        np.testing.assert_allclose(er[b, :k], o["ev_real"][b, :k], rtol=1e-12, atol=1e-9)


def test_cfg2_minn_rtl_full_batch_exact(variant):
    B, T, Q = 4096, 1024, 64
    x = int12_batch(B, T, 2 * Q, 22)
    assert _lib.lib().ofs_rtl_plan(_lib.CI16, 2, T, Q) > 2000
    a = minn_rtl.minn_rtl_batched(x, Q, hysteresis=2)
    variant("EXACT", 0)
    g = minn_rtl.minn_rtl_batched(x, Q, hysteresis=2)
    variant("EXACT", None)
    for k in ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled", "energy_scaled",
              "metric_valid", "above_threshold", "n_events", "open_gate_start"):
        assert torch.equal(getattr(a, k), getattr(g, k)), k
    xi = x.cpu().numpy()
    xc = (xi[..., 0] + 1j * xi[..., 1]).astype(np.complex128)
    o = oracle_c.minn_rtl(xc, Q, minn_rtl.SMOOTH_SHIFT, minn_rtl.THRESH_VALUE, minn_rtl.THRESH_FRAC_BITS, 2, 0,
                          max_events=int(a.events.shape[1]), nthreads=16)
    for k in ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled", "energy_scaled"):
        assert np.array_equal(getattr(a, k).cpu().numpy(), o[k]), k
    assert np.array_equal(a.metric_valid.cpu().numpy(), o["metric_valid"].astype(bool))
    assert np.array_equal(a.above_threshold.cpu().numpy(), o["above_threshold"].astype(bool))
    n = a.n_events.cpu().numpy()
    assert np.array_equal(n, o["n_events"]) and np.array_equal(a.open_gate_start.cpu().numpy(), o["open_gate_start"])
    ev = a.events.cpu().numpy()
    for b in range(B):
        k = min(int(n[b]), ev.shape[1])
        assert np.array_equal(ev[b, :k], o["events"][b, :k])


def test_cfg4_fused_shard_every_stream_vs_oracle():
    B, T, N = 32768, 4096, 2048
    x = synth.make_aa_batch(B, T, N // 2, seed=4, device="cuda")
    assert _lib.lib().ofs_win_plan(4, _lib.C64, _lib.FP32, 1, T, N) == 42        # sc_minn kernel, E = 4
    (Mm, Pm, Rm), (Ms, Ps, Rs) = combined_sc_min.sc_minn_streaming_metrics_batched(x, N)
    assert Ms.shape == (B, T - N + 1)
    kP, kR, kM = EM.win_fast_k(4, 1)
    h = lambda t: t.cpu().numpy()                                                 # noqa: E731
    st = np.concatenate([oracle_c.sc_minn_check(h(x[lo:lo + 4096]), N, h(Ms[lo:lo + 4096]), h(Ps[lo:lo + 4096]),
                                                h(Rs[lo:lo + 4096]), h(Mm[lo:lo + 4096]), h(Pm[lo:lo + 4096]),
                                                h(Rm[lo:lo + 4096]), kP, kR, kM, nthreads=16)
                         for lo in range(0, B, 4096)])
    worst = dict(zip(oracle_c.SC_MINN_STATS, st.max(axis=0)))
    print("cfg4 every stream:", {k: float(f"{v:.3g}") for k, v in worst.items()})
    assert not np.isnan(st).any()
    assert worst["comb_max_dM"] <= 1e-6 and worst["minn_max_dM_rel1"] <= 1e-6          # north star
    for k in ("comb_dM_over_bound", "comb_dP_over_bound", "comb_dR_over_bound", "minn_dM_over_bound",
              "minn_dP_over_bound", "minn_dR_over_bound"):
        assert worst[k] <= 1.0, k


def test_cfg3_detect_only_full_batch_vs_oracle(variant):
    """The headline batch with P/R/M not stored (SURVEY §8d detect-only): every stream's events
    against the C oracle (oracle/parity.py: exact except stated near-ties; CFO angle <= 1e-6).
    The detect-only kernel runs 4 samples per lane per row with fp32 row scans (aa_fast.hip
    pick_e_do, scan32); the M the classifier needs comes from the storing kernel forced to the
    same row width and scan precision, i.e. the same arithmetic, so both calls' events are
    identical too."""
    import parity
    B, T, L = 65536, 1024, 512
    x = synth.headline_batch(B, T, L, seed=777)
    variant("FAST_E", 4)
    variant("FAST_SCAN", 32)
    full = sync_aa.aa_detect_streaming_batched(x, L, outputs=("M",), max_events=8)
    variant("FAST_E", None)
    variant("FAST_SCAN", None)
    det = sync_aa.aa_detect_streaming_batched(x, L, outputs=(), max_events=8)
    assert torch.equal(full.n_events, det.n_events)
    k = int(min(det.n_events.max(), 8))
    live = sync_aa.live_events(det.n_events, k)
    assert torch.equal(full.ev_int[:, :k][live], det.ev_int[:, :k][live])
    assert torch.equal(full.ev_real[:, :k][live], det.ev_real[:, :k][live])
    o = oracle_c.aa_detect(x.cpu().numpy(), L, max_events=8, nthreads=16)
    r = parity.classify_aa(full.M.cpu().numpy().astype(np.float64), det.n_events.cpu().numpy(),
                           det.ev_int.cpu().numpy(), det.ev_real.cpu().numpy(), o["P"], o["M"], o["n_events"],
                           o["ev_int"], o["ev_real"], L)
    print("detect-only parity:", r)
    assert r["mismatch"] == 0 and r["cfo_over_tol"] == 0 and r["events_engine"] == r["events_oracle"]


def test_cfg5_full_batch_every_sequence_vs_oracle():
    B, N = 1 << 20, 4096
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.empty((B, N), dtype=torch.complex64, device="cuda")
    for i in range(0, B, 1 << 17):                       # 32 GiB, generated in chunks
        x[i:i + (1 << 17)] = torch.randn((1 << 17, N), dtype=torch.complex64, device="cuda", generator=g)
    sym = torch.from_numpy(O.pss_symbol(N).astype(np.complex64)).cuda()
    x[::97] += 4.0 * sym                                                 # some windows carry the PSS
    idx, t, e = O.zc_template()
    assert _lib.lib().ofs_zc_freq_plan(_lib.C64, _lib.FP32, N, N, 0) == 3
    m = zc_freq.compute_frequency_metric_batched(x, idx, t, e, N=N, cp=0)
    assert m.shape == (B, 1) and m.dtype == torch.float32
    mh = m.cpu().numpy()
    assert float(mh[::97].min()) > 0.5
    eps = EM.zc_win_eps(N)
    CH = 1 << 16
    st = np.concatenate([oracle_c.zc_freq_check(x[lo:lo + CH].cpu().numpy(), N, 0, idx, t, e, mh[lo:lo + CH], eps,
                                                6.0, nthreads=16) for lo in range(0, B, CH)])
    print(f"cfg5 every sequence: max |dm| = {st[:, 0].max():.3g}, max |dm|/bound = {st[:, 1].max():.3g} "
          f"(eps = {eps:.3g}), oracle metric max {st[:, 2].max():.3f}")
    assert not np.isnan(st).any()
    assert st[:, 1].max() <= 1.0                        # error model 2 (worst case, Higham)
    assert st[:, 0].max() <= 1e-6                        # north star: float metric within 1e-6
