"""Shared check of fp32 sync_aa results against the fp64 oracle (tests only): metric / sums
within tolerance and EVERY event exact under oracle/parity.py's stated near-tie criterion."""
import numpy as np

import ofdm_oracle as O
import parity


def relerr(a, b):
    s = max(1.0, float(np.max(np.abs(b)))) if np.size(b) else 1.0
    return float(np.max(np.abs(np.asarray(a) - b))) / s if np.size(b) else 0.0


def check_fp32_batch(out, x, L, threshold=0.15, hysteresis=128, sample_rate=15.36e6, oracle=None):
    """out: AABatchResult (device), x: host [B, n_ant, T] complex64 samples the engine saw.
    oracle: optional list of per-stream (P, R, M, valid, ev_int, ev_real) (default: computed)."""
    B, _, T = x.shape
    M_g = out.M.cpu().numpy().astype(np.float64)
    P_g, R_g = out.P.cpu().numpy(), out.R.cpu().numpy()
    n_g = out.n_events.cpu().numpy()
    Emax = max(int(n_g.max(initial=0)), 1)
    assert out.ev_int.shape[1] >= Emax, "event buffer too small for the check"
    ei_g, er_g = out.ev_int.cpu().numpy()[:, :Emax], out.ev_real.cpu().numpy()[:, :Emax]
    P_o = np.zeros((B, T), np.complex128)
    M_o = np.zeros((B, T))
    n_o = np.zeros(B, np.int32)
    ei_o = np.zeros((B, Emax, 4), np.int64)
    er_o = np.zeros((B, Emax, 4))
    for b in range(B):
        if oracle is None:
            Pr, Rr, Mr, vr, ei, er = O.aa_detect(x[b].astype(np.complex128), L, threshold, hysteresis, sample_rate)
        else:
            Pr, Rr, Mr, vr, ei, er = oracle[b]
        assert np.max(np.abs(M_g[b] - Mr), initial=0) < 1e-6
        assert relerr(P_g[b], Pr) < 1e-5 and relerr(R_g[b], Rr) < 1e-5
        if out.valid is not None:
            assert np.array_equal(out.valid[b].cpu().numpy(), vr)
        P_o[b], M_o[b], n_o[b] = Pr, Mr, len(ei)
        k = min(len(ei), Emax)
        ei_o[b, :k], er_o[b, :k] = ei[:k], er[:k]
        assert np.array_equal(ei_g[b, :min(n_g[b], Emax), 3], ei_g[b, :min(n_g[b], Emax), 0] - 2 * L + 1)
    r = parity.classify_aa(M_g, n_g, ei_g, er_g, P_o, M_o, n_o, ei_o, er_o, L, threshold, hysteresis)
    assert r["mismatch"] == 0 and r["cfo_over_tol"] == 0, r
    return r
