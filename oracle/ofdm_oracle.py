"""CPU oracle: a NumPy restatement of the reference's timing-metric + CFO hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker
(or as the timed CPU baseline).  The product path (``ofdm-sync-math_amd/``) never
imports it and has no CPU fallback.

Parity pinning: every function here is checked against golden vectors produced by the
reference itself (``tests/golden/make_golden.py`` imports /root/reference and runs it)
and against the reference's own fixtures ``docs/detector_test_vector.csv`` /
``docs/detector_cfo_test_vector.csv`` (tests/test_oracle_golden.py).

The restatement is written in prefix-sum form (float64 ``cumsum``) rather than the
reference's per-sample recursion; for float inputs the two agree to ~1e-12 relative,
for integer-valued inputs (int12 ADC samples) they are bit-identical because every
partial sum is an exactly representable integer (< 2**53).  The gate/peak state
machines are restated as literal loops, statement for statement.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "aa_metric", "aa_events", "aa_detect",
    "sc_metric", "comb_sc_metric", "minn_metric",
    "minn_rtl_metric", "detect_minn_rtl", "cp_cfo", "cp_cfo_robust", "cp_cfo_peak", "find_cp_start",
    "rx_backend",
    "park_metric", "zc_template", "zc_freq_metric", "pss_symbol", "matched_filter",
    "normalize_correlation", "zc_combined", "zc_streaming_detection", "detect_zc_peaks",
    "trailing_average", "plateau_end", "minn_peak", "sc_gate", "streaming_peak", "comb_minn_peak",
]


def _as2d(x, dtype=np.complex128):
    x = np.asarray(x)
    if x.ndim == 1:
        x = x[np.newaxis, :]
    return x.astype(dtype, copy=False)


def _pref(v):
    """Exclusive-at-zero prefix: p[i+1] = sum(v[:i+1]); p[0] = 0."""
    out = np.zeros(v.shape[:-1] + (v.shape[-1] + 1,), dtype=v.dtype)
    np.cumsum(v, axis=-1, out=out[..., 1:])
    return out


# ---------------------------------------------------------------------------------------
# sync_aa.aa_detect_streaming  (sync_aa.py:421-571)
# ---------------------------------------------------------------------------------------
def aa_metric(rx, L):
    """P[n], R[n], M[n], valid[n] of sync_aa.aa_detect_streaming (sync_aa.py:458-493).

    product[j] = x[j]*conj(x[j-L]) for j >= L, else 0          (DelayLine, :377-386, :466-469)
    P[n] = sum_{j=n-L+1..n} product[j] (window clipped at 0)      (RunningSum, :331-342)
    R[n] = sum_{j=n-L+1..n} |x[j]|^2                               (RunningSumReal, :355-365)
    valid[n] = n >= L                                              (filled == L, :338-342)
    M = min(|P|^2/R^2, 1) if valid and R > 1e-6*L else 0           (:486-493)
    """
    x = _as2d(rx)
    _, T = x.shape
    prod = np.zeros_like(x)
    if T > L:
        prod[:, L:] = x[:, L:] * np.conj(x[:, :-L])
    e = (x.real ** 2 + x.imag ** 2)
    Pp = _pref(prod.sum(axis=0))
    Ep = _pref(e.sum(axis=0))
    n = np.arange(T)
    lo = np.maximum(n - L + 1, 0)
    P = Pp[n + 1] - Pp[lo]
    R = Ep[n + 1] - Ep[lo]
    valid = n >= L
    M = np.zeros(T)
    ok = valid & (R > 1e-6 * L)
    M[ok] = np.minimum((np.abs(P[ok]) ** 2) / (R[ok] ** 2), 1.0)
    return P, R, M, valid


def aa_events(P, M, valid, L, threshold=0.15, hysteresis=128, sample_rate=15.36e6):
    """Gate/peak/CFO state machine, literal restatement of sync_aa.py:495-568.

    Returns (ints[k,4] = peak_index, gate_start, gate_end, frame_start,
             reals[k,4] = P_re, P_im, M_at_peak, cfo_hz).
    """
    T = len(M)
    ints, reals = [], []
    gate_open = False
    gate_start = peak_index = low_count = 0
    peak_P = 0j
    peak_mag = 0.0

    def emit(end):
        cfo = np.angle(peak_P) * sample_rate / (2 * np.pi * L)
        ints.append((peak_index, gate_start, end, peak_index - 2 * L + 1))
        reals.append((peak_P.real, peak_P.imag, M[peak_index], cfo))

    for n in range(T):
        if not valid[n]:
            continue
        m = M[n]
        pm = np.abs(P[n]) ** 2
        if not gate_open:
            if m >= threshold:
                gate_open, gate_start, peak_index, peak_P, peak_mag, low_count = True, n, n, P[n], pm, 0
        else:
            if pm > peak_mag:
                peak_index, peak_P, peak_mag = n, P[n], pm
            if m >= threshold:
                low_count = 0
            else:
                low_count += 1
                if low_count >= hysteresis:
                    emit(n)
                    gate_open, peak_mag, low_count = False, 0.0, 0
    if gate_open:
        emit(T)
    return (np.array(ints, dtype=np.int64).reshape(-1, 4),
            np.array(reals, dtype=np.float64).reshape(-1, 4))


def aa_detect(rx, L=512, threshold=0.15, hysteresis=128, sample_rate=15.36e6):
    P, R, M, valid = aa_metric(rx, L)
    ints, reals = aa_events(P, M, valid, L, threshold, hysteresis, sample_rate)
    return P, R, M, valid, ints, reals


def aa_metric_loop(rx, L):
    """Literal per-sample form of sync_aa.py:458-493 (DelayLine :368-386, RunningSum :321-342,
    RunningSumReal :345-365 as ring buffers, one Python iteration per sample and antenna).

    Same complexity as the reference (the "literal-loop" CPU baseline of bench.py); values
    equal the reference's recursion bit for bit (same operation order, Python complex/float).
    """
    x = _as2d(rx)
    na, T = x.shape
    rows = [list(map(complex, x[a])) for a in range(na)]
    dl = [[0j] * L for _ in range(na)]
    pb = [[0j] * L for _ in range(na)]
    rb = [[0.0] * L for _ in range(na)]
    ps = [0j] * na
    rs = [0.0] * na
    ptr, filled = 0, 0
    P = np.zeros(T, np.complex128)
    R = np.zeros(T)
    M = np.zeros(T)
    valid = np.zeros(T, bool)
    floor_ = 1e-6 * L
    for n in range(T):
        P_sum, R_sum = 0j, 0.0
        ok = filled >= L                            # delay / window filled before this push
        for a in range(na):
            xn = rows[a][n]
            xd = dl[a][ptr]
            dl[a][ptr] = xn
            prod = xn * xd.conjugate() if ok else 0j
            ps[a] = ps[a] + prod - pb[a][ptr]
            pb[a][ptr] = prod
            pw = abs(xn) ** 2
            rs[a] = rs[a] + pw - rb[a][ptr]
            rb[a][ptr] = pw
            P_sum += ps[a]
            R_sum += rs[a]
        ptr = ptr + 1 if ptr + 1 < L else 0
        if filled < L:
            filled += 1
        P[n], R[n], valid[n] = P_sum, R_sum, ok
        if ok and R_sum > floor_:
            M[n] = min(abs(P_sum) ** 2 / R_sum ** 2, 1.0)
    return P, R, M, valid


def aa_detect_loop(rx, L=512, threshold=0.15, hysteresis=128, sample_rate=15.36e6):
    """aa_detect in the reference's literal streaming form (aa_metric_loop + aa_events)."""
    P, R, M, valid = aa_metric_loop(rx, L)
    ints, reals = aa_events(P, M, valid, L, threshold, hysteresis, sample_rate)
    return P, R, M, valid, ints, reals


# ---------------------------------------------------------------------------------------
# sc.sc_streaming_metric (sc.py:42-78) and combined_sc_min.schmidl_cox_streaming_metric
# (combined_sc_min.py:116-164)
# ---------------------------------------------------------------------------------------
def _sc_common(rx, N, both_halves):
    x = _as2d(rx)
    _, T = x.shape
    half = N // 2
    out_len = T - N + 1
    if half == 0 or out_len <= 0:
        return np.zeros(0), np.zeros(0, np.complex128), np.zeros(0)
    if N != 2 * half:
        raise ValueError("symbol length must be even (halves of equal length)")
    # P(d) = sum_{k<half} x[d+k] conj(x[d+half+k])
    prod = (x[:, :-half] * np.conj(x[:, half:])).sum(axis=0)          # index j = d+k
    Pp = _pref(prod)
    Ep = _pref((x.real ** 2 + x.imag ** 2).sum(axis=0))
    d = np.arange(out_len)
    P = Pp[d + half] - Pp[d]
    if both_halves:
        R = Ep[d + N] - Ep[d]                                         # combined_sc_min.py:154
    else:
        R = Ep[d + N] - Ep[d + half]                                  # sc.py:61
    M = (np.abs(P) ** 2) / (np.maximum(R, 1e-12) ** 2)
    return M, P, R


def sc_metric(rx, N):
    """sc.sc_streaming_metric with sc.N_FFT == N (sc.py:42-78)."""
    return _sc_common(rx, N, both_halves=False)


def comb_sc_metric(rx, N):
    """combined_sc_min.schmidl_cox_streaming_metric(rx, symbol_len=N) (combined_sc_min.py:116-164)."""
    return _sc_common(rx, N, both_halves=True)


# ---------------------------------------------------------------------------------------
# Minn metric: minn.minn_streaming_metric (minn.py:59-112), _parameterized (minn.py:697-751),
# combined_sc_min.minn_streaming_metric (combined_sc_min.py:60-113)
# ---------------------------------------------------------------------------------------
def minn_metric(rx, N):
    x = _as2d(rx)
    _, T = x.shape
    Q = N // 4
    out_len = T - N + 1
    if out_len <= 0:
        return np.zeros(0), np.zeros(0, np.complex128), np.zeros(0)
    if Q == 0:
        z = np.zeros(out_len)
        return z, np.zeros(out_len, np.complex128), z.copy()
    # C(d) = sum_{k<Q} x[d+k] conj(x[d+Q+k]);  P = C(d) + C(d+2Q)
    prod = (x[:, :-Q] * np.conj(x[:, Q:])).sum(axis=0)
    Cp = _pref(prod)
    Ep = _pref((x.real ** 2 + x.imag ** 2).sum(axis=0))
    d = np.arange(out_len)
    P = (Cp[d + Q] - Cp[d]) + (Cp[d + 3 * Q] - Cp[d + 2 * Q])
    R = Ep[d + 4 * Q] - Ep[d + Q]
    M = np.clip(P.real, 0.0, None) ** 2 / (np.maximum(R, 1e-12) ** 2)
    return M, P, R


# ---------------------------------------------------------------------------------------
# minn_rtl.minn_rtl_streaming_metric (minn_rtl.py:667-733) + detect_minn_rtl (:750-825)
# ---------------------------------------------------------------------------------------
def minn_rtl_metric(rx, Q, smooth_shift, threshold_value, threshold_frac_bits, smooth_mode="float"):
    """Closed form of the _antenna_path pipeline (minn_rtl.py:583-652), summed over branches.

    prod[j] = Re(x[j] conj(x[j-Q])) for j >= Q else 0     (_DelayLine fill phase, :524-542)
    C[i] = sum_{j=i-Q+1..i} prod[j];  E[i] = sum |x[j]|^2   (_RunningSum, :558-580)
    corr_recent = C[i]   (i >= Q-1), corr_previous = C[i-Q]   (i >= 2Q-1)
    energy: E[i] (i >= Q-1), E[i-Q] (i >= 2Q-1), E[i-2Q] (i >= 3Q-1); registers hold 0 before
    taps_valid = i >= 3Q-1.
    smooth_mode "float": the float64 IIR of minn_rtl.py:706-715 (bit-exact restatement);
    "floor": the integer floor-shift IIR of ref/minn_preamble_detector.sv:288-296.
    """
    x = _as2d(rx)
    _, T = x.shape
    if Q <= 0:
        raise ValueError("quarter_len must be positive.")
    prod = np.zeros(x.shape)
    if T > Q:
        prod[:, Q:] = x[:, :-Q].real * x[:, Q:].real + x[:, :-Q].imag * x[:, Q:].imag
    pw = x.real * x.real + x.imag * x.imag
    Cp = _pref(prod.sum(axis=0))
    Ep = _pref(pw.sum(axis=0))
    i = np.arange(T)
    lo = np.maximum(i - Q + 1, 0)
    C = Cp[i + 1] - Cp[lo]
    E = Ep[i + 1] - Ep[lo]

    def delayed(a, k, start):
        out = np.zeros(T)
        m = i >= start
        out[m] = a[i[m] - k]
        return out

    corr_total = delayed(C, 0, Q - 1) + delayed(C, Q, 2 * Q - 1)
    energy_total = delayed(E, 0, Q - 1) + delayed(E, Q, 2 * Q - 1) + delayed(E, 2 * Q, 3 * Q - 1)
    valid = i >= 3 * Q - 1
    corr_positive = np.maximum(corr_total, 0.0)
    smooth = np.zeros(T)
    s = 0.0
    if smooth_mode == "float":
        denom = 1 << max(0, smooth_shift)
        for k in range(T):
            if valid[k]:
                if smooth_shift == 0:
                    s = corr_positive[k]
                else:
                    s += (corr_positive[k] - s) / denom
            smooth[k] = s
    elif smooth_mode == "floor":
        si = 0
        cpi = corr_positive.astype(np.int64)
        for k in range(T):
            if valid[k]:
                si = int(cpi[k]) if smooth_shift == 0 else si + ((int(cpi[k]) - si) >> smooth_shift)
            smooth[k] = si
    else:
        raise ValueError(smooth_mode)
    corr_scaled = smooth * (1 << threshold_frac_bits)
    energy_scaled = np.zeros(T) if threshold_value == 0 else energy_total * float(threshold_value)
    above = valid & (corr_scaled >= energy_scaled)
    return dict(corr_total=corr_total, corr_positive=corr_positive, smooth_metric=smooth,
                energy_total=energy_total, corr_scaled=corr_scaled, energy_scaled=energy_scaled,
                metric_valid=valid, above_threshold=above)


def detect_minn_rtl(corr_positive, above, valid, hysteresis, timing_offset):
    """Literal restatement of minn_rtl.detect_minn_rtl (minn_rtl.py:750-825).

    Returns (events[k,4] = peak_index, detected_index, seg_start, seg_end,
             segments[s,2], gate_mask).
    """
    T = len(corr_positive)
    segs, evs = [], []
    gate_open = False
    gate_start = None
    peak_value = 0.0
    peak_index = low = 0
    hyst_limit = hysteresis - 1 if hysteresis > 0 else 0
    for idx in range(T):
        if not valid[idx]:
            continue
        v = corr_positive[idx]
        if not gate_open:
            if above[idx]:
                gate_open, gate_start, peak_value, peak_index, low = True, idx, v, idx, 0
        else:
            if v >= peak_value:
                peak_value, peak_index = v, idx
            if above[idx]:
                low = 0
            else:
                closing = hysteresis == 0 or low == hyst_limit
                if not closing:
                    low += 1
                if closing:
                    seg = (gate_start if gate_start is not None else idx, idx + 1)
                    segs.append(seg)
                    evs.append((peak_index, peak_index + timing_offset, seg[0], seg[1]))
                    gate_open, gate_start, peak_value, low = False, None, 0.0, 0
    if gate_open and gate_start is not None:
        segs.append((gate_start, T))
    mask = np.zeros(T, dtype=bool)
    for a, b in segs:
        mask[a:b] = True
    return (np.array(evs, dtype=np.int64).reshape(-1, 4),
            np.array(segs, dtype=np.int64).reshape(-1, 2), mask)


# ---------------------------------------------------------------------------------------
# core.estimate_cfo_from_cp (core.py:179-196)
# ---------------------------------------------------------------------------------------
def cp_cfo(rx, start, n_fft, cp_len, fs_hz):
    x = _as2d(rx)
    a = x[:, start:start + cp_len]
    b = x[:, start + n_fft:start + n_fft + cp_len]
    P = np.sum(a * np.conj(b))
    return float(-np.angle(P) * fs_hz / (2 * np.pi * n_fft)), complex(P)


# ---------------------------------------------------------------------------------------
# CP-correlation searches (core.py:199-336)
# ---------------------------------------------------------------------------------------
def _cp_window(x, d, n_fft, w):
    return np.sum(x[:, d:d + w] * np.conj(x[:, d + n_fft:d + n_fft + w]))


def cp_cfo_robust(rx, est, n_fft, cp_len, fs_hz, span=None, win_len=None):
    """core.estimate_cfo_from_cp_robust (core.py:199-231): angle of sum_d P_win(d) over
    d in [max(0, est-span), min(T-(N+win), est+span)); empty range -> estimate_cfo_from_cp at
    est with min(cp_len, win) samples (:222-223)."""
    x = _as2d(rx)
    T = x.shape[1]
    span = cp_len // 2 if span is None else int(max(0, span))
    win = cp_len // 2 if win_len is None else int(max(1, win_len))
    lo, hi = max(0, est - span), min(T - (n_fft + win), est + span)
    if hi <= lo:
        return cp_cfo(x, est, n_fft, min(cp_len, win), fs_hz)[0]
    P = 0j
    for d in range(lo, hi):
        P += _cp_window(x, d, n_fft, win)
    return float(-np.angle(P) * fs_hz / (2 * np.pi * n_fft))


def cp_cfo_peak(rx, est, n_fft, cp_len, fs_hz, span=None):
    """core.estimate_cfo_from_cp_peak_with_index (core.py:271-303; estimate_cfo_from_cp_peak
    :234-268 is its first element): first d maximising |P_cp(d)| (strict >) in the search
    range, CFO from P_cp(d); empty range -> (estimate_cfo_from_cp at est, est)."""
    x = _as2d(rx)
    T = x.shape[1]
    span = cp_len // 2 if span is None else int(max(0, span))
    lo, hi = max(0, est - span), min(T - (n_fft + cp_len), est + span)
    if hi <= lo:
        return cp_cfo(x, est, n_fft, cp_len, fs_hz)[0], int(est)
    best, bmag, bd = 0j, -1.0, lo
    for d in range(lo, hi):
        P = _cp_window(x, d, n_fft, cp_len)
        m = float(np.abs(P))
        if m > bmag:
            best, bmag, bd = P, m, d
    return float(-np.angle(best) * fs_hz / (2 * np.pi * n_fft)), int(bd)


def find_cp_start(rx, est, n_fft, cp_len, search_half=1024):
    """core.find_cp_start_via_corr (core.py:306-336)."""
    x = _as2d(rx)
    T = x.shape[1]
    lo, hi = max(0, est - search_half), min(T - (n_fft + cp_len), est + search_half)
    if hi <= lo:
        return int(est)
    bd, bv = lo, -1.0
    for d in range(lo, hi):
        v = float(np.abs(_cp_window(x, d, n_fft, cp_len)))
        if v > bv:
            bv, bd = v, d
    return int(bd)


# ---------------------------------------------------------------------------------------
# receiver back-end chain of sc.run_simulation (sc.py:274-311) over core.py helpers
# ---------------------------------------------------------------------------------------
def rx_backend(rx, pilot_start, data_start, n_fft, cp, fs, bins, pilot_used, data_used, cfo=None):
    """cfo = estimate_cfo_from_cp at the pilot CP (core.py:179-196) unless given; rx_eff =
    branch mean of apply_cfo(rx, -cfo) (core.py:123-138); y = fftshift(fft(window))[(N/2+k)%N]
    (ofdm_fft_used, core.py:171-176); h = y_p/(pilot+1e-9) (:339-341); slope/sto from the
    unwrapped phase of h (:443-469, abscissa = bins); xhat = y_d/(h+1e-9) (:344-345);
    gain = vdot(xhat, ref)/(vdot(xhat, xhat)+1e-12) (:357-362); evm (:365-370)."""
    x = _as2d(rx)
    if cfo is None:
        cfo = cp_cfo(x, pilot_start, n_fft, cp, fs)[0]
    n = np.arange(x.shape[1], dtype=float)
    tone = np.exp(1j * 2 * np.pi * (-cfo) * n / fs)
    eff = np.mean(x * tone[np.newaxis, :], axis=0)
    k = np.asarray(bins)

    def used(s):
        spec = np.fft.fftshift(np.fft.fft(eff[s + cp:s + cp + n_fft], n=n_fft))
        return spec[(n_fft // 2 + k) % n_fft]

    h = used(pilot_start) / (np.asarray(pilot_used) + 1e-9)
    phi = np.unwrap(np.angle(h))
    kz = k.astype(float) - np.mean(k.astype(float))
    pz = phi - np.mean(phi)
    slope = float(np.sum(kz * pz) / (float(np.sum(kz * kz)) + 1e-12))
    xhat = used(data_start) / (h + 1e-9)
    ref = np.asarray(data_used)
    g = np.vdot(xhat, ref) / (np.vdot(xhat, xhat) + 1e-12)
    xa = xhat * g
    evm = float(np.sqrt(np.mean(np.abs(xa - ref) ** 2) / np.mean(np.abs(ref) ** 2)))
    return dict(cfo=float(cfo), h=h, xa=xa, gain=complex(g), evm=evm, evm_db=float(20 * np.log10(evm + 1e-12)),
                slope=slope, sto=float(-slope * n_fft / (2 * np.pi)))


# ---------------------------------------------------------------------------------------
# park.park_streaming_metric (park.py:64-114)
# ---------------------------------------------------------------------------------------
def park_metric(rx, N):
    """(ds, M, P, E) of park.park_streaming_metric with park.N_FFT = N.

    half = N//2; ds = [half, T-half-1]                               (:76-96)
    P(d) = sum_br sum_{k<half} x[d-k] * x[d+k]   (no conjugate)      (:103-107)
    E(d) = sum_br sum_{k<half} |x[d+k]|^2                            (:108)
    M = |P|^2 / max(E, 1e-12)^2                                      (:112-113)
    Vectorised over d, looping over k (same products, summed in k order per branch).
    """
    x = _as2d(rx)
    nb, T = x.shape
    half = N // 2
    if half == 0 or T < 2 * half + 1:
        return (np.zeros(0, dtype=int), np.zeros(0), np.zeros(0, np.complex128), np.zeros(0))
    ds = np.arange(half, T - half)
    P = np.zeros(ds.size, np.complex128)
    E = np.zeros(ds.size)
    for b in range(nb):
        xb = x[b]
        Pb = np.zeros(ds.size, np.complex128)
        for k in range(half):
            Pb += xb[ds - k] * xb[ds + k]
        e = np.abs(xb) ** 2
        Eb = (_pref(e)[ds + half] - _pref(e)[ds])
        P += Pb
        E += Eb
    M = np.abs(P) ** 2 / np.maximum(E, 1e-12) ** 2
    return ds, M, P, E


# ---------------------------------------------------------------------------------------
# zc_freq.compute_frequency_metric (zc_freq.py:62-99) + make_pss_frequency_template (:54-59)
# ---------------------------------------------------------------------------------------
def zc_template(length=62, root=25):
    """(bin_indices, template_bins, energy): centered +-1..+-length/2 (core.py:13-18), ZC
    root/length sequence exp(-j*pi*r*n*(n+1)/len) (zc_freq.py:37-39)."""
    half = length // 2
    idx = np.concatenate((np.arange(-half, 0), np.arange(1, half + 1)))
    n = np.arange(length)
    t = np.exp(-1j * np.pi * root * n * (n + 1) / length)
    return idx, t, float(np.sum(np.abs(t) ** 2))


def zc_freq_metric(rx, N, cp, bin_indices, template_bins, template_energy):
    """metric[off] for off in [0, T-(N+cp)]: window x[off+cp : off+cp+N] per branch,
    bins = fftshift(fft(window))[(N/2 + idx) % N] == fft(window)[idx % N];
    metric = |sum_br vdot(t, bins)|^2 / max(E_t * sum_br sum |bins|^2, 1e-12).
    The 62 DFT bins are evaluated as a direct DFT (matrix product) instead of a full FFT;
    identical mathematics, agreement ~1e-13 relative.  Raises ValueError when too short (:76-78).
    """
    x = _as2d(rx)
    nb, T = x.shape
    noff = T - (N + cp) + 1
    if noff <= 0:
        raise ValueError("Received stream is shorter than a single OFDM symbol.")
    k = np.asarray(bin_indices) % N
    W = np.exp(-2j * np.pi * np.outer(np.arange(N), k) / N)            # [N][62]
    t = np.asarray(template_bins, np.complex128)
    corr = np.zeros(noff, np.complex128)
    en = np.zeros(noff)
    CH = 2048
    for b in range(nb):
        win = np.lib.stride_tricks.sliding_window_view(x[b, cp:], N)[:noff]
        for o0 in range(0, noff, CH):
            bins = win[o0:o0 + CH] @ W
            corr[o0:o0 + CH] += bins @ np.conj(t)
            en[o0:o0 + CH] += np.sum(np.abs(bins) ** 2, axis=1)
    return np.abs(corr) ** 2 / np.maximum(template_energy * en, 1e-12)


# ---------------------------------------------------------------------------------------
# ZC matched filter: zc_v2.py:244-271 and the inline combiner of zc.py:106-126
# ---------------------------------------------------------------------------------------
def pss_symbol(N, length=62, root=25):
    """zc_v2.build_pss_symbol(include_cp=False) / zc.build_pss_symbol(False) for N_FFT = N:
    ZC on centered bins, ifft(ifftshift(.)), scaled to unit mean power (core.py:21-40)."""
    idx, t, _ = zc_template(length, root)
    spec = np.zeros(N, np.complex128)
    spec[(N // 2 + idx) % N] = t
    td = np.fft.ifft(np.fft.ifftshift(spec))
    p = np.mean(np.abs(td) ** 2)
    return td if p == 0 else td / np.sqrt(p)


def matched_filter(x, ref):
    """np.convolve(x, conj(ref[::-1]), 'full') (zc_v2.py:244-254)."""
    return np.convolve(np.asarray(x, np.complex128), np.conj(np.asarray(ref)[::-1]))


def _window_energy_full(x, n):
    """np.convolve(|x|^2, ones(n), 'full') as a prefix difference (length T+n-1)."""
    e = np.abs(np.asarray(x)) ** 2
    p = _pref(e)
    T = e.size
    i = np.arange(T + n - 1)
    return p[np.minimum(i + 1, T)] - p[np.maximum(i + 1 - n, 0)]


def normalize_correlation(corr, x, ref):
    """corr / (sqrt(E_ref) * sqrt(max(window_energy, 1e-12))) (zc_v2.py:257-271)."""
    ref = np.asarray(ref)
    e = _window_energy_full(x, ref.size)
    return corr / (np.sqrt(np.sum(np.abs(ref) ** 2)) * np.sqrt(np.maximum(e, 1e-12)))


def zc_combined(rx, ref):
    """zc.py:106-126: sum_br conv(x, conj(ref[::-1])) / (|ref| * sqrt(max(sum_br E, 0) + 1e-12))."""
    x = _as2d(rx)
    ref = np.asarray(ref)
    num = sum(matched_filter(b, ref) for b in x)
    pw = sum(_window_energy_full(b, ref.size) for b in x)
    return num / (np.sqrt(np.sum(np.abs(ref) ** 2)) * np.sqrt(np.maximum(pw, 0.0) + 1e-12))


def zc_streaming_detection(corr_mag, window_size, thresh_value, thresh_frac_bits, min_corr_mag):
    """zc_v2.zc_streaming_detection (zc_v2.py:300-346), RunningSum (:219-238) restated
    literally (sequential float64 add/subtract, valid once W samples have been pushed)."""
    c = np.asarray(corr_mag, np.float64)
    n = c.size
    W = max(1, int(window_size))
    local = np.zeros(n)
    valid = np.zeros(n, bool)
    acc = 0.0
    for i in range(n):
        if i >= W:
            acc = acc + c[i] - c[i - W]
            valid[i] = True
        else:
            acc = acc + c[i]
        local[i] = acc
    cs = c * float(1 << thresh_frac_bits)
    ts = local * float(thresh_value)
    above = valid & (cs >= ts) & (c >= min_corr_mag)
    return dict(corr_mag=c, local_sum=local, corr_scaled=cs, thresh_scaled=ts,
                above_threshold=above, metric_valid=valid)


def detect_zc_peaks(corr_mag, above, valid, reference_length, hysteresis):
    """Literal restatement of zc_v2.detect_zc_peaks (zc_v2.py:374-446).

    Returns (events[k,4] = peak_index, gate_start, gate_end, detected_start,
             peak_values[k], gate_mask)."""
    n = len(corr_mag)
    mask = np.zeros(n, bool)
    evs, vals = [], []
    gate_open = False
    gate_start = peak_index = low = 0
    peak_value = 0.0
    hyst_limit = max(0, hysteresis - 1)
    for i in range(n):
        if not valid[i]:
            continue
        v = corr_mag[i]
        if not gate_open:
            if above[i]:
                gate_open, gate_start, peak_index, peak_value, low = True, i, i, v, 0
        else:
            mask[i] = True
            if v > peak_value:
                peak_value, peak_index = v, i
            if above[i]:
                low = 0
            elif hysteresis == 0 or low >= hyst_limit:
                evs.append((peak_index, gate_start, i, max(0, peak_index - reference_length + 1)))
                vals.append(peak_value)
                gate_open, peak_value, low = False, 0.0, 0
            else:
                low += 1
    if gate_open:
        evs.append((peak_index, gate_start, n, max(0, peak_index - reference_length + 1)))
        vals.append(peak_value)
        mask[gate_start:n] = True
    return np.array(evs, np.int64).reshape(-1, 4), np.array(vals, np.float64), mask


# ---------------------------------------------------------------------------------------
# Detection post-processing: turns a metric stream into a timing decision.
# ---------------------------------------------------------------------------------------
def trailing_average(x, win):
    """minn._trailing_average (minn.py:115-128) == combined_sc_min._trailing_average
    (combined_sc_min.py:167-180): the running sum adds x[i] and drops x[i-win], divided by the
    number of samples seen (capped at win).  Literal float64 recursion."""
    x = np.asarray(x, dtype=float)
    if win <= 1:
        return x.copy()
    y = np.empty_like(x)
    acc = 0.0
    for i in range(x.size):
        acc += x[i]
        if i >= win:
            acc -= x[i - win]
        y[i] = acc / (win if i >= win - 1 else i + 1)
    return y


def _runs(mask):
    """[start, end) of the True runs of a boolean mask, in order."""
    m = np.concatenate(([False], np.asarray(mask, bool), [False]))
    d = np.flatnonzero(m[1:] != m[:-1])
    return list(zip(d[0::2], d[1::2]))


def _py_slice(n, start, stop):
    """Indices of a[start:stop] for len(a) == n (Python slice semantics, step 1)."""
    return range(n)[start:stop]


def plateau_end(M, cp_len, lookahead=None, smooth_win=8):
    """sc.find_plateau_end_from_metric (sc.py:81-146).  Returns (index, branch, Ms) with branch
    1 = first drop below 95 % of the smoothed maximum (:106-114), 2 = right edge of the earliest
    run >= max(8, cp/2) above 60 % (:117-133), 3 = slope fallback (:136-146), 4 = fallback with
    an empty drop window (:142-143), 0 = empty metric."""
    M = np.asarray(M, dtype=float)
    if M.size == 0:
        return 0, 0, M.copy()
    L = (cp_len // 4) if lookahead is None else int(max(1, lookahead))
    w = max(1, smooth_win)
    Ms = np.convolve(M, np.ones(w, dtype=float) / w, mode="same")
    center = int(np.argmax(Ms))
    post_hi = min(Ms.size, center + cp_len)
    if post_hi > center + 1:
        below = np.flatnonzero(Ms[center:post_hi] <= 0.95 * float(Ms[center]))
        if below.size > 0:
            return int(center + below[0]), 1, Ms
    min_run = max(8, cp_len // 2)
    peak = float(np.max(Ms))
    if peak > 0:
        for s, e in _runs(Ms >= 0.6 * peak):
            if e - s >= min_run:
                return int(e - 1), 2, Ms
    lo = max(0, center - cp_len)
    hi = min(Ms.size - L - 1, center + cp_len)
    win_idx = _py_slice(Ms.size, lo, hi)
    ahead_idx = _py_slice(Ms.size, lo + L, hi + L)
    window, ahead = Ms[list(win_idx)], Ms[list(ahead_idx)]
    drop = window - ahead              # numpy broadcasting rules (raises on a length mismatch)
    if drop.size == 0:
        return center, 4, Ms
    return lo + int(np.argmax(drop)) + (L // 2), 3, Ms


def _bounds(n, search_bounds):
    if search_bounds is None:
        return 0, n
    start, end = max(0, search_bounds[0]), min(n, search_bounds[1])
    return (0, n) if start >= end else (start, end)


def minn_peak(M, smooth_win=8, gate_threshold=0.5, search_bounds=None):
    """minn.find_minn_peak (minn.py:131-205): (peak_idx, gate_mask, Ms).  The gate is the
    LONGEST run of Ms >= gate_threshold * max(Ms) (earliest on ties), cut to the search bounds;
    an empty gate falls back to the global argmax.  Raises ValueError like the reference."""
    M = np.asarray(M, dtype=float)
    if M.size == 0:
        raise ValueError("Minn metric is empty")
    Ms = trailing_average(np.maximum(M, 0.0), max(1, smooth_win))
    mx = float(np.max(Ms))
    if mx <= 0.0:
        raise ValueError("Minn metric did not produce a positive peak")
    gate = np.zeros(M.size, bool)
    best = None
    for s, e in _runs(Ms >= gate_threshold * mx):
        if best is None or e - s > best[1] - best[0]:
            best = (s, e)
    if best is not None:
        gate[best[0]:best[1]] = True
    lo, hi = _bounds(M.size, search_bounds)
    if search_bounds is not None:
        b = np.zeros(M.size, bool)
        b[lo:hi] = True
        gate &= b
    if not gate.any():
        pk = int(np.argmax(Ms))
        gate = np.zeros(M.size, bool)
        gate[pk] = True
        return pk, gate, Ms
    idx = np.flatnonzero(gate)
    return int(idx[int(np.argmax(Ms[idx]))]), gate, Ms


def sc_gate(M_sc, threshold=0.6):
    """The S&C gate of combined_sc_min.run_simulation (combined_sc_min.py:337-358): normalise by
    the maximum, threshold, seed with the argmax if nothing passes.  Returns (mask, span)."""
    M_sc = np.asarray(M_sc, dtype=float)
    mx = float(np.max(M_sc))
    mask = (M_sc / mx >= threshold) if mx > 0 else (M_sc >= threshold)
    if not mask.any():
        mask = np.zeros(M_sc.size, bool)
        mask[int(np.argmax(M_sc))] = True
    idx = np.flatnonzero(mask)
    return mask, (int(idx[0]), int(idx[-1]) + 1)


def streaming_peak(metric, gate_mask):
    """combined_sc_min._streaming_peak_detector (combined_sc_min.py:183-209): first argmax
    (strict >) over the FIRST run of the gate; None if the gate never opens."""
    best_idx, best_val, active = None, -np.inf, False
    for i, v in enumerate(metric):
        if gate_mask[i]:
            if not active:
                active, best_val, best_idx = True, v, i
            elif v > best_val:
                best_val, best_idx = v, i
        elif active:
            return best_idx
    return best_idx


def comb_minn_peak(M, smooth_win, gate_mask, search_bounds=None):
    """combined_sc_min.find_minn_peak (combined_sc_min.py:212-259)."""
    M = np.asarray(M, dtype=float)
    if M.size == 0:
        return 0
    mask = np.asarray(gate_mask, bool).copy()
    if mask.shape[0] != M.shape[0]:
        raise ValueError("gate_mask must match metric length")
    if search_bounds is not None:
        lo, hi = _bounds(M.size, search_bounds)
        b = np.zeros(M.size, bool)
        b[lo:hi] = True
        mask &= b
    if not mask.any():
        raise ValueError("Minn peak detector received empty gate region")
    Ms = trailing_average(np.maximum(M, 0.0), max(1, smooth_win))
    return streaming_peak(Ms, mask)


# ---------------------------------------------------------------------------------------
# the back-end helpers one by one (core.py:123-138, 171-176, 339-370, 443-469) and
# sync_aa.quantize_adc (sync_aa.py:263-291)
# ---------------------------------------------------------------------------------------
def apply_cfo(x, cfo, fs):
    """core.py:123-138: x * exp(i 2 pi cfo n / fs), one tone for every branch of a 2-D x."""
    x = np.asarray(x)
    n = np.arange(x.shape[-1], dtype=float)
    return x * np.exp(1j * 2 * np.pi * cfo * n / fs)


def fft_used(sym, N, bins):
    """core.py:171-176: fftshift(fft(sym, n=N))[(N/2 + k) % N]."""
    spec = np.fft.fftshift(np.fft.fft(sym, n=N))
    return spec[(N // 2 + np.asarray(bins)) % N]


def cdiv_eps(y, d, eps):
    """core.py:339-341 / :344-345: y / (d + eps)."""
    return np.asarray(y) / (np.asarray(d) + eps)


def remove_common_phase(x, ref=None):
    """core.py:348-354."""
    cpe = np.angle(np.mean(x)) if ref is None else np.angle(np.vdot(ref, x) / (np.vdot(ref, ref) + 1e-12))
    return x * np.exp(-1j * cpe), float(cpe)


def align_complex_gain(x, ref, eps=1e-12):
    """core.py:357-362."""
    g = np.vdot(x, ref) / (np.vdot(x, x) + eps)
    return x * g, g


def evm_rms_db(x, ref):
    """core.py:365-370."""
    e = float(np.sqrt(np.mean(np.abs(x - ref) ** 2) / np.mean(np.abs(ref) ** 2)))
    return e, float(20 * np.log10(e + 1e-12))


def phase_slope(h, bins, N):
    """core.py:443-469 with abscissa = the centred subcarrier indices `bins`."""
    if h.size == 0:
        return 0.0, 0.0
    k = np.asarray(bins, dtype=np.float64)
    phi = np.unwrap(np.angle(h.astype(np.complex128)))
    kz, pz = k - float(np.mean(k)), phi - float(np.mean(phi))
    slope = float(np.sum(kz * pz) / (float(np.sum(kz * kz)) + 1e-12))
    return slope, float(-slope * N / (2.0 * np.pi))


def quantize_adc(samples, full_scale, bits=12):
    """sync_aa.py:263-291 (numpy's own promotion decides float32 vs float64)."""
    levels = 2 ** (bits - 1)

    def q(v):
        v = np.clip(v / full_scale, -1.0, 1.0 - 1.0 / levels)
        return np.round(v * levels) / levels * full_scale
    return q(samples.real) + 1j * q(samples.imag)
