"""GPU parity of the streaming fp32 fast path for the S&C / combined S&C / Minn window
metrics (csrc/win_fast.hip) against the CPU oracle (fp64), through the C ABI.

Tolerance (fp32 path, complex64 input): every output of every stream within the fp32 error
model of tests/error_models.py (model 1: |dP| <= kP·u·Σ|x_i||x_i+lag| + u|P|, |dR| <= kR·u·R,
and their first-order propagation into M), evaluated per sample from the oracle's fp64 values;
the measured maximum of |error| / bound is printed.  On streams without a quiet/loud step
M is also within the north-star 1e-6 (absolute for M <= 1, relative above: the S&C-with-second-
half-R and Minn metrics are not bounded by 1).  The dispatch is asserted to be the fast kernel.
"""
import numpy as np
import pytest

import error_models as EM
import ofdm_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import _lib, sc, combined_sc_min, minn, synth  # noqa: E402

KIND = {"sc": 1, "comb": 2, "minn": 3}
ORACLE = {"sc": O.sc_metric, "comb": O.comb_sc_metric, "minn": O.minn_metric}


def run(kind, x, N):
    if kind == "sc":
        return sc.sc_streaming_metric_batched(x, N)
    if kind == "comb":
        return combined_sc_min.schmidl_cox_streaming_metric_batched(x, N)
    return minn.minn_streaming_metric_batched(x, N)


def m_ok(m, mo, tol=1e-6):
    return bool(np.all(np.abs(m - mo) <= tol * np.maximum(1.0, np.abs(mo))))


STRESS = {3: "quiet span before a loud one", 4: "quiet span after a loud one"}
# stress streams (a 60 dB step inside the window) are fp32-conditioned: a random-phase window
# sum cancels by ~sqrt(W) against Σ|terms|, which the model's S_abs carries


def check_model(kind, xh, N, M, P, R, Mo, Po, Ro, north_star=True):
    """Every output within error model 1; returns max |error| / bound over M, P, R."""
    bM, bP, bR = EM.window_model(kind, xh, N, Po, Ro, Mo)
    rM = np.abs(M.astype(np.float64) - Mo) / bM
    rP = np.abs(P.astype(np.complex128) - Po) / bP
    rR = np.abs(R.astype(np.float64) - Ro) / bR
    worst = float(max(rM.max(initial=0), rP.max(initial=0), rR.max(initial=0)))
    assert worst <= 1.0, (kind, float(rM.max()), float(rP.max()), float(rR.max()))
    if north_star:
        assert m_ok(M, Mo)
    return worst


@pytest.mark.parametrize("kind", ["sc", "comb", "minn"])
@pytest.mark.parametrize("N,T", [(2048, 4096), (1024, 1024), (1024, 3000), (512, 700), (256, 1024),
                                 (4096, 6000), (2048, 2048), (1024, 3001), (512, 701), (2048, 4097)])
def test_window_fast_path_vs_oracle(kind, N, T):
    plan = _lib.lib().ofs_win_plan(KIND[kind], _lib.C64, _lib.FP32, 1, T, N)
    # Minn N=256 (Q=64) is below the fast kernel's 128-sample row: general engine
    assert (plan == 0) if (kind == "minn" and N == 256) else (plan > 0), plan
    B = 6
    x = synth.make_aa_batch(B, T, min(N // 2 if kind != "minn" else N // 4, 1024), seed=N + T, device="cuda")
    x[3, :, : T // 3] *= 1e-3                      # quiet span before a loud one
    x[4, :, T // 2:] *= 1e-3                       # and after one
    M, P, R = run(kind, x, N)
    assert M.dtype == torch.float32 and M.shape == (B, T - N + 1)
    xh = x.cpu().numpy().astype(np.complex128)
    worst = 0.0
    for b in range(B):
        Mo, Po, Ro = ORACLE[kind](xh[b], N)
        worst = max(worst, check_model(kind, xh[b], N, M[b].cpu().numpy(), P[b].cpu().numpy(), R[b].cpu().numpy(),
                                       Mo, Po, Ro, north_star=b not in STRESS))
    print(f"{kind} N={N} T={T}: max |err|/bound = {worst:.3g}")


def test_window_fast_path_covers_cfg4():
    L = _lib.lib()
    assert L.ofs_win_plan(2, _lib.C64, _lib.FP32, 1, 4096, 2048) > 0
    assert L.ofs_win_plan(3, _lib.C64, _lib.FP32, 1, 4096, 2048) > 0
    assert L.ofs_win_plan(1, _lib.C64, _lib.FP32, 2, 4096, 2048) > 0       # 2 branches: fast too
    assert L.ofs_win_plan(1, _lib.C64, _lib.FP32, 3, 4096, 2048) == 0      # 3 branches: general
    assert L.ofs_win_plan(1, _lib.C128, _lib.FP64, 1, 4096, 2048) == 0     # fp64: general


@pytest.mark.parametrize("N,T", [(2048, 4096), (1024, 1024), (512, 1500), (256, 800), (2048, 2100),
                                 (2048, 4001), (512, 1501), (1024, 1025)])
def test_fused_sc_minn_vs_oracle(N, T):
    """combined_sc_min's two metrics from the fused one-pass kernel (cfg4 shape first)."""
    plan = _lib.lib().ofs_win_plan(4, _lib.C64, _lib.FP32, 1, T, N)
    assert (plan == 0) if N == 256 else (plan > 0), plan     # Q=64 < one 128-sample row
    B = 6
    x = synth.make_aa_batch(B, T, min(N // 2, 1024), seed=N + 3 * T, device="cuda")
    x[3, :, T // 2:] *= 1e-3
    (Mm, Pm, Rm), (Ms, Ps, Rs) = combined_sc_min.sc_minn_streaming_metrics_batched(x, N)
    xh = x.cpu().numpy().astype(np.complex128)
    worst = 0.0
    for b in range(B):
        for kind, (M, P, R), f in (("minn", (Mm, Pm, Rm), O.minn_metric), ("comb", (Ms, Ps, Rs), O.comb_sc_metric)):
            Mo, Po, Ro = f(xh[b], N)
            worst = max(worst, check_model(kind, xh[b], N, M[b].cpu().numpy(), P[b].cpu().numpy(),
                                           R[b].cpu().numpy(), Mo, Po, Ro, north_star=b not in STRESS))
    print(f"fused N={N} T={T}: max |err|/bound = {worst:.3g}")


def test_fused_sc_minn_general_fallback_fp64():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, 2, 900)) + 1j * rng.standard_normal((2, 2, 900))
    (Mm, Pm, Rm), (Ms, Ps, Rs) = combined_sc_min.sc_minn_streaming_metrics_batched(torch.from_numpy(x).cuda(), 256)
    for b in range(2):
        Mo, _, _ = O.minn_metric(x[b], 256)
        np.testing.assert_allclose(Mm[b].cpu().numpy(), Mo, rtol=1e-9, atol=1e-12)
        Mo, _, _ = O.comb_sc_metric(x[b], 256)
        np.testing.assert_allclose(Ms[b].cpu().numpy(), Mo, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("kind", ["sc", "comb", "minn", "fused"])
@pytest.mark.parametrize("N,T", [(2048, 4096), (1024, 3000), (512, 900), (1024, 3001)])
def test_fast_paths_two_branches_vs_oracle(kind, N, T):
    """Two receive branches summed inside the streaming fast kernels (the reference's 2-D input,
    e.g. combined_sc_min.run_simulation on cir1[:2]): same tolerances as one branch."""
    code = {"sc": 1, "comb": 2, "minn": 3, "fused": 4}[kind]
    assert _lib.lib().ofs_win_plan(code, _lib.C64, _lib.FP32, 2, T, N) > 0
    B = 5
    x = synth.synth_batch(synth.faded_base(min(N // 2, 1024), "cir1", (0, 1)), B, T, seed=N + T)
    xh = x.cpu().numpy().astype(np.complex128)
    if kind == "fused":
        (Mm, Pm, Rm), (Ms, Ps, Rs) = combined_sc_min.sc_minn_streaming_metrics_batched(x, N)
        outs = [("minn", Mm, Pm, Rm), ("comb", Ms, Ps, Rs)]
    else:
        M, P, R = run(kind, x, N)
        outs = [(kind, M, P, R)]
    worst = 0.0
    for k, M, P, R in outs:
        for b in range(B):
            Mo, Po, Ro = ORACLE[k](xh[b], N)
            worst = max(worst, check_model(k, xh[b], N, M[b].cpu().numpy(), P[b].cpu().numpy(), R[b].cpu().numpy(),
                                           Mo, Po, Ro))
    print(f"{kind} 2 branches N={N} T={T}: max |err|/bound = {worst:.3g}")
