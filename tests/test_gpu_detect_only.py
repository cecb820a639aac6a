"""Detect-only mode of the sync_aa detector (8 B/sample + per-stream events): with
P/R/M/valid not requested the kernels skip those stores and keep the events on chip.  The
events must be identical to the ones of the full call on every dispatch plan (fp32 fast path,
int12 integer-exact path, general engine with fused events); the general engine's multi-tile
plan still gets P/M buffers from the mirror.  Exact equality: same kernel, same arithmetic (the
register-staged fp32 detect-only kernel runs 4 samples per lane per row with fp32 row scans,
aa_fast.hip pick_e_do / scan32, so its full call is compared at that row width and scan precision:
variant FAST_E=4, variant FAST_SCAN=32; with variant FAST_SCAN_DO=64 it equals the fp64-scan storing kernel)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import _lib, synth, sync_aa  # noqa: E402


def _batch(kind, B, T, L):
    x = synth.make_aa_batch(B, T, L, seed=99, device="cuda")
    if kind == "c64":
        return x
    if kind == "c128":
        return x.to(torch.complex128)
    s = 2046.0 / float(x.abs().amax())
    re = torch.clamp(torch.round(x.real * s), -2048, 2047).to(torch.int16)
    im = torch.clamp(torch.round(x.imag * s), -2048, 2047).to(torch.int16)
    return torch.stack([re, im], dim=-1).contiguous()


@pytest.mark.parametrize("kind,T,L,plan_lo,plan_hi", [("c64", 1024, 512, 1000, 2000), ("ci16", 1024, 128, 2000, 3000),
                                                       ("c128", 1024, 512, 3000, 4000),
                                                       ("c128", 3000, 256, 3000, 4000), ("c128", 9000, 512, 3000, 4000),
                                                       ("c64", 4096, 512, 1100, 1200), ("c64", 5315, 256, 1100, 1200),
                                                       ("c64", 9000, 100, 2, 2)])
def test_detect_only_events_equal_full(kind, T, L, plan_lo, plan_hi, variant):
    B = 512
    x = _batch(kind, B, T, L)
    b = _lib.as_batch(x, batched=True)
    plan = _lib.lib().ofs_aa_plan(b.fmt, _lib.resolve_precision(b, None), 1, T, L)
    assert plan_lo <= plan <= plan_hi
    reg = 1000 <= plan < 1100                      # register-staged fp32 kernel: DO arithmetic
    for scan in ("32", "64") if reg else ("",):
        if reg:
            variant("FAST_E", 4)
            variant("FAST_SCAN", int(scan))
            variant("FAST_SCAN_DO", int(scan))
        full = sync_aa.aa_detect_streaming_batched(x, L)
        variant("FAST_E", None)
        variant("FAST_SCAN", None)
        det = sync_aa.aa_detect_streaming_batched(x, L, outputs=())
        variant("FAST_SCAN_DO", None)
        assert det.P is None and det.M is None and det.R is None
        assert torch.equal(full.n_events, det.n_events)
        assert int(full.n_events.sum()) > B // 4
        E = min(full.ev_int.shape[1], det.ev_int.shape[1])
        mask = (torch.arange(E, device="cuda")[None, :] < torch.clamp(full.n_events, max=E)[:, None])
        assert torch.equal(full.ev_int[:, :E][mask], det.ev_int[:, :E][mask])
        assert torch.equal(full.ev_real[:, :E][mask], det.ev_real[:, :E][mask])


def test_default_detect_only_vs_default_full_near_threshold():
    """The two DEFAULT calls on the fp32 fast path use different arithmetic (storing kernel: fp64
    row scans, 2 samples per lane; detect-only: fp32 row scans, 4 per lane), so their events may
    differ - but only at decisions the reference itself makes on a near-tie.  Streams whose [A][A]
    peak metric sits at the threshold (SNR ~ -2 dB: M ~ (S/(S+N))^2 ~ 0.15): both calls are exact
    against the C oracle under oracle/parity.py's criterion, and every stream where the two calls
    disagree holds an oracle flag tie (|M_o - thr| <= 1e-6) or a peak tie (|P_o|^2 at the two peaks
    within 1e-5 relative)."""
    import oracle_c
    import parity
    B, T, L, thr = 4096, 1024, 256, 0.15
    rng = np.random.default_rng(2024)
    a = (rng.choice([-1.0, 1.0], (B, L)) + 1j * rng.choice([-1.0, 1.0], (B, L))) / np.sqrt(2)
    snr = 10 ** (rng.uniform(-3.2, -0.8, B) / 10)
    x = (rng.standard_normal((B, T)) + 1j * rng.standard_normal((B, T))) / np.sqrt(2)
    off = rng.integers(0, T - 2 * L, B)
    for b in range(B):
        x[b, off[b]:off[b] + 2 * L] += np.sqrt(snr[b]) * np.tile(a[b], 2)
    x = x.astype(np.complex64)[:, None, :]
    xd = torch.from_numpy(x).cuda()
    E = 8
    full = sync_aa.aa_detect_streaming_batched(xd, L, outputs=("M",), max_events=E)
    det = sync_aa.aa_detect_streaming_batched(xd, L, outputs=(), max_events=E)
    o = oracle_c.aa_detect(x, L, max_events=E, nthreads=16)
    r = parity.classify_aa(full.M.cpu().numpy().astype(np.float64), full.n_events.cpu().numpy(),
                           full.ev_int.cpu().numpy(), full.ev_real.cpu().numpy(), o["P"], o["M"], o["n_events"],
                           o["ev_int"], o["ev_real"], L, thr)
    assert r["mismatch"] == 0 and r["cfo_over_tol"] == 0, r
    nf, nd = full.n_events.cpu().numpy(), det.n_events.cpu().numpy()
    ef, ed = full.ev_int.cpu().numpy(), det.ev_int.cpu().numpy()
    near = np.abs(o["M"] - thr) <= 1e-6
    near[:, :L] = False
    differ = 0
    for b in range(B):
        k = min(nf[b], E)
        if nf[b] == nd[b] and np.array_equal(ef[b, :k], ed[b, :k]):
            continue
        differ += 1
        if near[b].any():
            continue
        assert nf[b] == nd[b] and np.array_equal(ef[b, :k, 1:3], ed[b, :k, 1:3]), b     # same gates
        pm = np.abs(o["P"][b]) ** 2
        for j in range(k):
            p1, p2 = int(ef[b, j, 0]), int(ed[b, j, 0])
            assert abs(pm[p1] - pm[p2]) <= 1e-5 * max(pm[p1], pm[p2]), (b, j, p1, p2)
    print(f"near-threshold batch: full vs oracle {r}; default detect-only differs from the full call on "
          f"{differ} of {B} streams (all at stated ties); events per stream {nf.mean():.2f}")
    assert differ <= B // 50
