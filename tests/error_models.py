"""fp32 error models of the engine's single-precision fast paths (test infrastructure).

Every fp32 parity test derives its tolerance from one of these models instead of a fixed
number, and prints the measured error next to the bound.  u = 2^-24 is the fp32 unit roundoff;
inputs are complex64 on both sides (the oracle promotes the same samples to fp64), so input
rounding is not an error source.

1. Window sums (win_fast.hip, sc_minn_pk_kernel: S&C / combined S&C / Minn; E samples per lane,
   NB branches).  A window sum S = wh + (xh + f[e]) + suffix is built from: the lagged products
   in fp32 (2u per component, NB branches accumulated: NB - 1 more adds), in-lane forward /
   backward partials (at most E - 1 adds), the fp64 lane scan and row totals (exact to fp32
   resolution) rounded to fp32 three times (in-row prefix, row remainder, rows inside the
   window), the retained suffix (1 add) and the final 3 adds.  Per real component
   |dS| <= (E + 8 + NB)·u·Σ|terms|, so for the complex P
       |dP| <= kP·u·S_abs + u·|P|,   kP = sqrt(2)·(E + 8 + NB),   S_abs = Σ |x_i|·|x_i+lag|,
   R (non-negative terms, up to 4 windows added): |dR| <= kR·u·R, kR = E + 11 + NB,
   and the metric M = c²/R² (c = |P| or max(Re P, 0); fma, mul, v_rcp_f32 1 ulp, mul):
       |dM| <= 2·(c/R)·(bP/R) + (bP/R)² + 2·M·bR/R + kM·u·M,   kM = 6.
   For combined S&C, S_abs <= R/2 (Cauchy-Schwarz) and M <= 1/4, so the bound is below
   (sqrt(M)·kP/2 + 2M·kR + kM·M)·u <= 5e-7 at E = 4: the north-star 1e-6 holds for every input.
2. FFT-based zc_freq metric (zc_win kernels: fp32 radix-2 column FFTs of R = N/64 points with
   fp32-rounded twiddles, then fp64 twiddled column sums per bin; rocFFT leg: an fp32 FFT of all
   log2(N) stages).  Normwise relative FFT error (Higham, Accuracy and Stability of Numerical
   Algorithms, Thm 24.2): eps <= stages·eta, eta = mu + gamma_4·(sqrt(2) + mu) ~ (1 + 4·sqrt(2))·u
   with mu = u the twiddle error.  The column sums in fp64 add no fp32 error; 2 stages are added
   for the fp32 products / gather.  With rho = ||db||/||b|| <= eps·sqrt(N)·||w||/||b|| (Parseval)
   and m = |<T, b>|²/(E_t·||b||²) over the nb·62 gathered bins:
       |dm| <= 2·(sqrt(nb·m) + m)·rho + (nb + 1)·rho² + kM·u·m.
   (oracle_zc_freq_check evaluates it per window from the fp64 bins.)
3. Park fp32 (corr.hip park_kernel<fp32>): every output's P(d) = Σ_br Σ_{k<N/2} x[d-k]·x[d+k] is one
   fp32 chain of 2 FMAs per term and component (park_mac), so per component
   |dP| <= gamma_{2·h·nb}·Σ (|b.x f.x| + |b.y f.y|) <= 2·h·nb·u·S_abs (Higham Eq. 3.5, first order;
   |b.x f.x| + |b.y f.y| <= |b|·|f|), h = N/2, S_abs = Σ |x[d-k]|·|x[d+k]|; for the complex P
   |dP| <= sqrt(2)·(2·h·nb + 2)·u·S_abs.  E (non-negative terms): one chain of 2 FMAs per term plus
   at most OPT + 2 = 10 adds of the shared-window split: |dE| <= (2·h·nb + 10)·u·E.  M = |P|²/E²
   as in model 1 (kM = 6).
"""
from __future__ import annotations

import math

import numpy as np

U32 = 2.0 ** -24
ETA = (1.0 + 4.0 * math.sqrt(2.0)) * U32          # per radix-2 stage (complex butterfly + twiddle)


def win_fast_k(E: int, NB: int = 1):
    """(kP, kR, kM) of model 1 for a window kernel with E samples per lane and NB branches."""
    return math.sqrt(2.0) * (E + 8 + NB), float(E + 11 + NB), 6.0


def zc_win_eps(N: int) -> float:
    """Model 2, fused window-FFT kernel: fp32 column FFTs of N/64 points (+2 stages)."""
    return (math.log2(max(N // 64, 2)) + 2) * ETA


def rocfft_eps(N: int) -> float:
    """Model 2, rocFFT leg: all log2(N) stages in fp32 (+2)."""
    return (math.log2(N) + 2) * ETA


def park_bounds(x: np.ndarray, N: int):
    """Model 3 for one stream x[nb, T] (complex128): per-output (bP, bE, S_abs, E) of Park fp32."""
    x = np.atleast_2d(x)
    nb, T = x.shape
    h = N // 2
    ds = np.arange(h, T - h)
    s = np.zeros(ds.size)
    e = np.zeros(ds.size)
    for br in range(nb):
        ax = np.abs(x[br])
        for k in range(h):
            s += ax[ds - k] * ax[ds + k]
        e += np.convolve(ax ** 2, np.ones(h))[ds + h - 1]       # Σ_{k<h} |x[d+k]|²
    return math.sqrt(2.0) * (2 * h * nb + 2) * U32 * s, (2 * h * nb + 10) * U32 * e


def metric_bound(c, R, M, bP, bR, kM: float = 6.0):
    """First-order bound of M = c²/R² given |dc| <= bP, |dR| <= bR (models 1 and 3)."""
    Rm = np.maximum(R, 1e-12)
    p = bP / Rm
    return 2.0 * (c / Rm) * p + p * p + 2.0 * M * (bR / Rm) + kM * U32 * M + 1e-300


def _win_abs(ax, lag, W, nout):
    """Σ_{k<W} ax[d+k]·ax[d+k+lag] for d < nout (fp64 prefix sums of non-negative terms)."""
    p = np.concatenate(([0.0], np.cumsum(ax[:-lag] * ax[lag:])))
    d = np.arange(nout)
    return p[d + W] - p[d]


def window_model(kind: str, x: np.ndarray, N: int, P, R, M, E: int = 4):
    """Model 1 for one stream x[nb, T] (complex128) and the oracle's P, R, M of `kind`
    ("sc", "comb", "minn"): per-output bounds (bM, bP, bR).  E = 4 is the widest lane
    (win_fast.hip pick(): E in {2, 4}), so the bound covers every instantiation."""
    x = np.atleast_2d(x)
    nb, T = x.shape
    nout = T - N + 1
    kP, kR, kM = win_fast_k(E, nb)
    S = np.zeros(nout)
    for br in range(nb):
        ax = np.abs(x[br])
        if kind in ("sc", "comb"):
            S += _win_abs(ax, N // 2, N // 2, nout)
        else:
            Q = N // 4
            s = _win_abs(ax, Q, Q, T - Q + 1 - Q)               # windows starting at any d' <= T-2Q
            S += s[:nout] + s[2 * Q:2 * Q + nout]
    P, R, M = np.asarray(P), np.asarray(R), np.asarray(M)
    bP = kP * U32 * S + U32 * np.abs(P)
    bR = kR * U32 * R
    c = np.maximum(P.real, 0.0) if kind == "minn" else np.abs(P)
    return metric_bound(c, R, M, bP, bR, kM), bP, bR
