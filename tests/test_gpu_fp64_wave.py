"""The fp64 wave-per-stream sync_aa path for complex128 input (aa_exact_kernel<OFS_C128>, plan
3000 + 10*E + MR, any T): the numpy drop-in's arithmetic (sync_aa.py:421-571 in float64).  Checked
against the CPU oracle and against the general LDS engine (variant EXACT=0 routes the same call
there) on ragged lengths, one and two antennas, every supported L, and a loud burst next to a
quiet window.

Tolerances (written here, as for every fp64 path): P, R within 1e-11 of the stream maximum,
M within 1e-12 absolute; event indices exact against the general engine and the oracle."""
import numpy as np
import pytest

import ofdm_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import _lib, synth, sync_aa  # noqa: E402


def _streams(B, na, T, L, seed):
    if T < 2 * L:                                      # shorter than the preamble: plain noise
        g = torch.Generator(device="cuda").manual_seed(seed)
        return torch.randn((B, na, T), dtype=torch.complex128, device="cuda", generator=g)
    x = synth.make_aa_batch(B, T, L, seed=seed, device="cuda").to(torch.complex128)
    if na == 2:
        x2 = synth.make_aa_batch(B, T, L, seed=seed + 1, device="cuda").to(torch.complex128)
        x = torch.cat([x, x2], dim=1)
    return x.contiguous()


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-300, float(np.max(np.abs(b)))))


@pytest.mark.parametrize("T,L,na", [(1024, 512, 1), (1023, 512, 1), (3584, 1024, 1), (2024, 512, 2),
                                    (777, 128, 2), (300, 64, 1), (1, 64, 1), (130, 256, 1),
                                    (5315, 512, 2), (9000, 512, 1), (16384, 256, 1)])
def test_fp64_wave_vs_general_engine_and_oracle(T, L, na, variant):
    B = 64
    x = _streams(B, na, T, L, seed=T + L)
    assert _lib.lib().ofs_aa_plan(_lib.C128, _lib.FP64, na, T, L) > 3000
    got = sync_aa.aa_detect_streaming_batched(x, L)
    variant("EXACT", 0)
    assert _lib.lib().ofs_aa_plan(_lib.C128, _lib.FP64, na, T, L) in (1, 2)
    ref = sync_aa.aa_detect_streaming_batched(x, L)
    variant("EXACT", None)
    for name, tol in (("P", 1e-11), ("R", 1e-11)):
        a, b = getattr(got, name).cpu().numpy(), getattr(ref, name).cpu().numpy()
        assert _rel(a, b) <= tol, name
    np.testing.assert_allclose(got.M.cpu().numpy(), ref.M.cpu().numpy(), rtol=0, atol=1e-12)
    assert torch.equal(got.valid, ref.valid)
    assert torch.equal(got.n_events, ref.n_events)
    n = min(got.ev_int.shape[1], ref.ev_int.shape[1])
    for b in range(B):
        k = min(int(got.n_events[b]), n)
        assert torch.equal(got.ev_int[b, :k], ref.ev_int[b, :k])
        np.testing.assert_allclose(got.ev_real[b, :k].cpu().numpy(), ref.ev_real[b, :k].cpu().numpy(),
                                   rtol=1e-9, atol=1e-9)
    xh = x.cpu().numpy()
    for b in (0, B // 2, B - 1):
        Po, Ro, Mo, Vo = O.aa_metric(xh[b], L)
        assert _rel(got.P[b].cpu().numpy(), Po) <= 1e-11
        np.testing.assert_allclose(got.M[b].cpu().numpy(), Mo, rtol=0, atol=1e-12)


def test_fp64_wave_loud_burst_next_to_quiet_window():
    """60 dB step: a loud burst, then a quiet [A][A].  After the burst every formulation carries a
    residue of ~ulp(energy of the burst) in its window sums - the reference's RunningSum adds and
    subtracts the loud samples (sync_aa.py:331-365), the oracle and both GPU engines difference
    fp64 prefixes - so quiet-window metrics agree to ~1e-9 relative, not 1e-12: tolerance here
    1e-8 absolute on M (values up to 1), and the detection itself must be unaffected."""
    T, L, B = 2048, 256, 16
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((B, 1, T)) + 1j * rng.standard_normal((B, 1, T))) * 1e-3
    x[:, :, :600] *= 1e3
    pre = rng.standard_normal(L) + 1j * rng.standard_normal(L)
    x[:, 0, 1000:1000 + L] += 1e-2 * pre
    x[:, 0, 1000 + L:1000 + 2 * L] += 1e-2 * pre
    xd = torch.from_numpy(x).cuda()
    got = sync_aa.aa_detect_streaming_batched(xd, L)
    for b in range(B):
        Po, Ro, Mo, Vo = O.aa_metric(x[b], L)
        np.testing.assert_allclose(got.M[b].cpu().numpy(), Mo, rtol=0, atol=1e-8)
    assert float(got.M[:, 1000 + 2 * L - 1].min()) > 0.5
    assert int(got.n_events.min()) >= 1
