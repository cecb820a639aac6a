"""Full-batch parity of the fp32 [A][A] detector against the fp64 oracle, with near-tie
exemptions stated explicitly.

TEST / BASELINE INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg).

The reference's decisions (sync_aa.py:495-568) are comparisons of float64 values: above =
M[n] >= threshold (:512, :525) and the strict running maximum of |P|^2 in the gate (:519).
An fp32 engine reproduces every decision whose margin exceeds its rounding; a decision whose
margin is below it is a tie the two precisions may break differently.  Criterion:

* above flags: the engine's flag may differ from the oracle's only where the oracle's metric
  is within ``tol_m`` of the threshold (|M_o - thr| <= tol_m; tol_m = 1e-6 = the north-star
  metric tolerance, measured fp32 error ~1.5e-7).  Any other flag difference is a MISMATCH.
* gates: re-running the reference gate machine on the ORACLE's |P|^2 with the ENGINE's
  above flags must give exactly the engine's gate_start / gate_end / event count.
* peak: equal to the oracle's, or a tie: |P_o|^2 at the engine's peak >= (1 - tol_p) x the
  maximum of |P_o|^2 over the gate (tol_p = 1e-5: fp32 |P|^2 relative error at a gate peak,
  where |P| >= sqrt(thr)·R, is <= ~4e-6).
* CFO (peak equal): |angle(P_g) - angle(P_o)| <= tol_a rad (tol_a = 1e-6; the CFO is that
  angle x fs / (2 pi L)).

Streams are classified exact / flag_tie / peak_tie / mismatch; parity holds iff mismatch == 0.
"""
from __future__ import annotations

import numpy as np


def _events_from_flags(above, valid, pm, hyst):
    """sync_aa.py:495-568 gate machine with given above flags; peaks by the strict > running
    max of pm.  Returns list of (peak, gate_start, gate_end)."""
    T = len(above)
    ev = []
    gate_open, gs, pk, pmax, low = False, 0, 0, 0.0, 0
    for n in range(T):
        if not valid[n]:
            continue
        if not gate_open:
            if above[n]:
                gate_open, gs, pk, pmax, low = True, n, n, pm[n], 0
        else:
            if pm[n] > pmax:
                pk, pmax = n, pm[n]
            if above[n]:
                low = 0
            else:
                low += 1
                if low >= hyst:
                    ev.append((pk, gs, n))
                    gate_open, pmax, low = False, 0.0, 0
    if gate_open:
        ev.append((pk, gs, T))
    return ev


def classify_aa(M_g, n_g, ei_g, er_g, P_o, M_o, n_o, ei_o, er_o, L, threshold=0.15, hysteresis=128,
                tol_m=1e-6, tol_p=1e-5, tol_a=1e-6):
    """M_g [B,T] engine metric; n/ei/er engine and oracle events ([B], [B,E,4], [B,E,4]);
    P_o, M_o [B,T] oracle complex P and metric.  Returns a dict of counts and statistics."""
    B, T = M_g.shape
    E = min(ei_g.shape[1], ei_o.shape[1])
    valid = np.arange(T) >= L
    ab_g = (M_g >= threshold) & valid
    ab_o = (M_o >= threshold) & valid
    flag_diff = ab_g != ab_o
    amb = np.abs(M_o - threshold) <= tol_m
    hard_flag = (flag_diff & ~amb).any(axis=1)
    any_flag = flag_diff.any(axis=1)
    ne = np.minimum(n_g, E)
    same_n = n_g == n_o
    k = np.arange(E)[None, :]
    live = k < ne[:, None]
    ints_eq = np.all((ei_g[:, :E, :3] == ei_o[:, :E, :3]).all(axis=2) | ~live, axis=1) & same_n
    peak_eq = (ei_g[:, :E, 0] == ei_o[:, :E, 0]) & live & (k < np.minimum(n_o, E)[:, None])
    # event slots past n_events are never written by the engine (uninitialised buffers): the
    # angle is only formed where both sides hold a live event with the same peak
    rg = np.where(peak_eq[..., None], er_g[:, :E, :2], 1.0)
    ro = np.where(peak_eq[..., None], er_o[:, :E, :2], 1.0)
    dang = np.abs(np.angle(np.exp(1j * (np.arctan2(rg[..., 1], rg[..., 0]) - np.arctan2(ro[..., 1], ro[..., 0])))))
    cfo_err = np.where(peak_eq, dang, 0.0)
    exact = ints_eq & ~any_flag
    cls = np.full(B, "exact", dtype=object)
    stats = dict(flag_tie=0, peak_tie=0, mismatch=0)
    bad_streams = []
    for b in np.flatnonzero(~exact | hard_flag):
        if hard_flag[b]:
            cls[b] = "mismatch"
            stats["mismatch"] += 1
            bad_streams.append(int(b))
            continue
        pm = np.abs(P_o[b]) ** 2
        ev = _events_from_flags(ab_g[b], valid, pm, hysteresis)
        ok = len(ev) == n_g[b]
        tie_peak = False
        for j, (pk, gs, ge) in enumerate(ev[:E] if ok else []):
            if ei_g[b, j, 1] != gs or ei_g[b, j, 2] != ge:
                ok = False
                break
            pg = int(ei_g[b, j, 0])
            if pg != pk:
                hi = min(ge, T - 1)
                best = pm[gs:hi + 1].max()
                if not (gs <= pg <= hi and pm[pg] >= (1.0 - tol_p) * best):
                    ok = False
                    break
                tie_peak = True
        if not ok:
            cls[b] = "mismatch"
            bad_streams.append(int(b))
        elif tie_peak:
            cls[b] = "peak_tie"
        else:
            cls[b] = "flag_tie"
        stats[cls[b]] += 1
    cfo_bad = int((cfo_err > tol_a).sum())
    return dict(streams=int(B), exact=int((cls == "exact").sum()), flag_tie=stats["flag_tie"],
                peak_tie=stats["peak_tie"], mismatch=stats["mismatch"], events_engine=int(n_g.sum()),
                events_oracle=int(n_o.sum()), max_abs_err_M=float(np.max(np.abs(M_g - M_o))),
                max_cfo_angle_err_rad=float(cfo_err.max(initial=0.0)), cfo_over_tol=cfo_bad,
                first_mismatch_streams=bad_streams[:8],
                criterion=f"flags may differ only where |M_o-thr|<={tol_m:g}; gates exact under the engine's "
                          f"flags; peak within (1-{tol_p:g}) of the oracle max |P|^2; CFO angle <= {tol_a:g} rad")
