// aa_gate.h — gate / peak event machines streamed row by row inside a wave-per-stream kernel:
//   sync_aa   (sync_aa.py:495-568):   peak = FIRST argmax of |P|² in the gate (strict >),
//             events (peak, gate_start, gate_end, frame_start) + (P, M, CFO), an open gate closes
//             at T;   used by aa_fast.hip (fp32 values) and aa_exact.hip (fp64 values);
//   minn_rtl  (minn_rtl.py:750-825):  peak = LAST argmax of corr_positive (>=), events
//             (peak, peak + timing_offset, gate_start, gate_end + 1), an open gate is reported
//             as open_gate_start;  used by aa_exact.hip.
//
// Both machines have the same gate structure: the gate opens at an above-threshold sample when
// closed, any above sample resets the low counter, and it closes at the max(H, 1)-th consecutive
// non-above sample.  Closed form (ofdmsync.hip, aa_events): with prev(n) = last above position
// <= n, a gate closes at n iff prev(n) exists and n - prev(n) == max(H, 1); it opens at an above
// sample whose predecessor gap is >= max(H, 1); opens and closes alternate; the peak is the
// arg-extremum over [open, close].  Rows hold RL = 64·E samples, lane l owns samples
// RL·k + E·l + e.  Per row: prev-above by lane-serial + DPP max-scan, opens / closes by ballot
// (with H >= RL: from the row's first/last above bits alone, no scan); the per-gate
// arg-extremum is tracked per lane across rows and reduced over the wave once per event.
#pragma once
#include "ofs_common.h"

namespace ofs {

// gate machine variants (paired A/B builds): scan-free flags when H >= RL (template FF: on for
// the fp64 kernels and the detect-only fp32 kernel - 5-8 % there - off for the fp32 kernel that
// also stores P/R/M, where it measured 1-2 % slower); per-lane peak tracking reduced over the
// wave once per event instead of once per row (template DEFER; neutral on the headline, off
// for the complex128 kernel whose extra fp64 lane state cost it occupancy)
#ifndef OFS_GATE_FASTFLAGS
#define OFS_GATE_FASTFLAGS 1
#endif
#ifndef OFS_GATE_PRED
#define OFS_GATE_PRED 0
#endif
#ifndef OFS_GATE_NOINLINE_EMIT
#define OFS_GATE_NOINLINE_EMIT 0
#endif
#ifndef OFS_GATE_FFONLY
#define OFS_GATE_FFONLY 0
#endif
#ifndef OFS_GATE_DIAG
#define OFS_GATE_DIAG 0
#endif
#ifndef OFS_GATE_NOACC
#define OFS_GATE_NOACC 0
#endif
#ifndef OFS_GATE_DEFER
#define OFS_GATE_DEFER 1
#endif

constexpr int GATE_NOKEY = 1 << 20;      // row-relative keys
constexpr int ABS_NOKEY = 0x7fffffff;    // absolute sample indices

template <int E, class V, bool RTL = false, bool FF = true, bool DEFER = true>
struct AaRowGate {
    static constexpr int RL = 64 * E;
    int Hp, L, max_ev, toff;
    double thr, fs;
    int64_t* evi;
    double* evr;
    int carry_last, n_ev, ev_start, gate_open, bidx;
    V bpm, bpr, bpi, bm;

    __device__ __forceinline__ void init(int hyst, int L_, double thr_, double fs_, int max_ev_,
                                         int64_t* evi_, double* evr_, int toff_ = 0) {
        Hp = hyst > 1 ? hyst : 1;
        L = L_; max_ev = max_ev_; thr = thr_; fs = fs_; evi = evi_; evr = evr_; toff = toff_;
        carry_last = -1; n_ev = 0; ev_start = 0; gate_open = 0; bidx = 0;
        bpm = (V)-1; bpr = (V)0; bpi = (V)0; bm = (V)0;
        lane_reset();
    }

    // the record is wave-uniform: lanes 0..3 store the four int64 fields and lanes 4..7 the four
    // f64 fields, one store instruction per 32-byte record half (a lane-0 loop of 8-byte stores
    // cost ~450 B of write traffic per event, measured with WRITE_SIZE)
#if OFS_GATE_NOINLINE_EMIT
    __device__ __attribute__((noinline)) void emit(int lane, int gate_end) {
#else
    __device__ __forceinline__ void emit(int lane, int gate_end) {
#endif
        if (evi && n_ev < max_ev && lane < 8) {
            int64_t* ei = evi + (int64_t)n_ev * 4;
            if constexpr (RTL) {
                const int64_t f[4] = {bidx, (int64_t)bidx + toff, ev_start, (int64_t)gate_end + 1};
                if (lane < 4) ei[lane] = f[lane & 3];
            } else {
                double* er = evr + (int64_t)n_ev * 4;
                const int64_t f[4] = {bidx, ev_start, gate_end, (int64_t)bidx - 2 * L + 1};
                if (lane < 4) {
                    ei[lane] = f[lane & 3];
                } else {
                    // fp32 values: fp32 atan2 (P itself carries ~1e-6 relative error; the fp64 ocml
                    // atan2 is ~250 VALU per event), fp64 values: atan2
                    const double ang = sizeof(V) == 4 ? (double)fast_atan2f((float)bpi, (float)bpr)
                                                      : atan2((double)bpi, (double)bpr);
                    const double g[4] = {(double)bpr, (double)bpi, (double)bm, ang * fs / (2.0 * M_PI * (double)L)};
                    er[lane - 4] = g[lane & 3];
                }
            }
        }
        n_ev += 1;
    }

    // sync_aa row (all positions >= L): above = m >= threshold; m = metric, pm = |P|², pr/pi = P
    __device__ __forceinline__ void row(int lane, int k, int nb, int T, const V (&m)[E], const V (&pm)[E],
                                        const V (&pr)[E], const V (&pi)[E]) {
#if OFS_GATE_DIAG == 1              // diagnostic builds only (wrong events): no row work at all
        return;
#endif
        bool ab[E];
#pragma unroll
        for (int e = 0; e < E; ++e) ab[e] = (nb + e < T) && (double)m[e] >= thr;
#if OFS_GATE_DIAG == 2              // diagnostic builds only: the above ballots, nothing else
        uint64_t any = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) any |= __ballot(ab[e]);
        if (any) carry_last = RL * k;
        return;
#endif
        row_flags(lane, k, nb, T, ab, pm, pr, pi, m);
    }

    // per-lane running arg-extremum of the open gate: each lane keeps its best (value, absolute
    // index, payload) over the rows the gate has covered; the wave reduction runs once, when the
    // gate closes (first max / strict > for sync_aa, last max / >= for minn_rtl, as a global scan)
    V lv, lpr, lpi, lm;
    int lk;
    __device__ __forceinline__ void lane_reset() {
        lv = (V)-1; lpr = (V)0; lpi = (V)0; lm = (V)0;
        lk = RTL ? -1 : ABS_NOKEY;
    }
    __device__ __forceinline__ void accumulate(int lane, int k, int nb, int T, int lo, int hi, const V (&pm)[E],
                                               const V (&pr)[E], const V (&pi)[E], const V (&m)[E]) {
#if OFS_GATE_NOACC == 1             // diagnostic builds only (wrong peaks): no per-lane peak tracking
        return;
#endif
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int key = E * lane + e;
            const bool in = nb + e < T && key >= lo && key <= hi;
            const bool better = RTL ? (pm[e] >= lv) : (pm[e] > lv);
#if OFS_GATE_NOACC == 2             // diagnostic builds only (wrong payload): value + index tracked
            if (in && better) { lv = pm[e]; lk = RL * k + key; }
#else
            if (in && better) { lv = pm[e]; lk = RL * k + key; lpr = pr[e]; lpi = pi[e]; lm = m[e]; }
#endif
        }
    }
    // wave reduction of the lanes' running bests into the event's peak (kept if it beats the
    // peak so far under the machine's tie rule), then the lanes restart
#if OFS_GATE_NOINLINE_EMIT
    __device__ __attribute__((noinline)) void merge() {
#else
    __device__ __forceinline__ void merge() {
#endif
        const V vmax = wave_max(lv);
        const int kk = RTL ? wave_max_i(lv == vmax ? lk : -1) : wave_min(lv == vmax ? lk : ABS_NOKEY);
        const bool found = RTL ? (kk >= 0) : (kk != ABS_NOKEY);
        const bool take = RTL ? (vmax >= bpm) : (vmax > bpm);
        if (found && take) {
            const int ln = (kk % RL) / E;
            bpr = readlane(lpr, ln);
            bpi = readlane(lpi, ln);
            bm = readlane(lm, ln);
            bpm = vmax;
            bidx = kk;
        }
        lane_reset();
    }
    // a gate's samples within one row; OFS_GATE_DEFER = 0 reduces over the wave every row
    __device__ __forceinline__ void seg(int lane, int k, int nb, int T, int lo, int hi, const V (&pm)[E],
                                        const V (&pr)[E], const V (&pi)[E], const V (&m)[E]) {
        accumulate(lane, k, nb, T, lo, hi, pm, pr, pi, m);
        if (!(DEFER && OFS_GATE_DEFER)) merge();
    }
    __device__ __forceinline__ void open_at(int start) {
        gate_open = 1; ev_start = start; bpm = (V)-1; lane_reset();
    }

    // generic row: above flags given; pm = the value whose arg-extremum is the peak
    __device__ __forceinline__ void row_flags(int lane, int k, int nb, int T, const bool (&ab)[E],
                                              const V (&pm)[E], const V (&pr)[E], const V (&pi)[E],
                                              const V (&m)[E]) {
#if OFS_GATE_PRED
        if (FF && DEFER && OFS_GATE_DEFER && Hp >= RL) {
            // the scan-free machine with the common path predicated: the only branch left per row is
            // the (rare) gate close; opening, the carry and the per-lane peak tracking are selects
            int first = GATE_NOKEY, last = -1;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint64_t am = __ballot(ab[e]);
                const int f = am ? E * (int)__builtin_ctzll(am) + e : GATE_NOKEY;
                const int l = am ? E * (63 - (int)__builtin_clzll(am)) + e : -1;
                first = min(first, f);
                last = max(last, l);
            }
            const int base = RL * k;
            const int c = carry_last + Hp;
            if (carry_last >= 0 && c >= base && c < base + RL && c < T && c - base < first) {
                accumulate(lane, k, nb, T, gate_open ? 0 : -1, c - base, pm, pr, pi, m);
                merge();
                emit(lane, c);
                gate_open = 0;
            }
            const bool has = first != GATE_NOKEY;
            const bool opens = has && (carry_last < 0 || base + first - 1 - carry_last >= Hp);
            carry_last = has ? base + last : carry_last;
            ev_start = opens ? base + first : ev_start;
            bpm = opens ? (V)-1 : bpm;
            lv = opens ? (V)-1 : lv;
            lk = opens ? (RTL ? -1 : ABS_NOKEY) : lk;
            const int lo = opens ? first : (gate_open ? 0 : RL);    // RL: empty range (gate closed)
            gate_open = (opens || gate_open) ? 1 : 0;
            accumulate(lane, k, nb, T, lo, RL - 1, pm, pr, pi, m);
            return;
        }
#endif
        if (FF && OFS_GATE_FASTFLAGS && (OFS_GATE_FFONLY || Hp >= RL)) {
            // hysteresis at least one row: only the row's FIRST above sample can open a gate and
            // only carry_last + Hp can close one (before that first sample), so the machine runs
            // on the above ballots alone, in scalar registers - no prefix scan
            int first = GATE_NOKEY, last = -1;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint64_t am = __ballot(ab[e]);
                if (am) {
                    first = min(first, E * (int)__builtin_ctzll(am) + e);
                    last = max(last, E * (63 - (int)__builtin_clzll(am)) + e);
                }
            }
            const int base = RL * k;
            int seg_lo = gate_open ? 0 : -1;
            if (carry_last >= 0) {                                   // close at carry_last + Hp
                const int c = carry_last + Hp;
                if (c >= base && c < base + RL && c < T && c - base < first) {
                    seg(lane, k, nb, T, seg_lo, c - base, pm, pr, pi, m);
                    if (DEFER && OFS_GATE_DEFER) merge();
                    emit(lane, c);
                    gate_open = 0; seg_lo = -1;
                }
            }
            if (first != GATE_NOKEY) {
                const int f = base + first;
                if (carry_last < 0 || f - 1 - carry_last >= Hp) {   // open
                    open_at(f); seg_lo = first;
                }
                carry_last = base + last;
            }
            if (gate_open) seg(lane, k, nb, T, seg_lo, RL - 1, pm, pr, pi, m);
            return;
        }
#if OFS_GATE_FFONLY                 // diagnostic builds only (H >= one row assumed): no scan path
        return;
#endif
        int lane_last = -1;
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (ab[e]) lane_last = nb + e;
        const int W = max(wave_scan_max(lane_last, lane), carry_last);
        int run = wave_shr1(W, lane, carry_last);
        uint64_t Om[E], Cm[E];
        uint64_t any = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int n = nb + e;
            const int pe = run;
            if (ab[e]) run = n;
            const bool cl = (n < T) && run >= 0 && (n - run) == Hp;
            const bool op = ab[e] && (pe < 0 || (n - 1 - pe) >= Hp);
            Om[e] = __ballot(op);
            Cm[e] = __ballot(cl);
            any |= Om[e] | Cm[e];
        }
        carry_last = readlane(W, 63);

        int seg_lo = gate_open ? 0 : -1;
        if (any) {
            int pos = -1;
            while (true) {
                int key = GATE_NOKEY, is_open = 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int q = pos - e;
                    const int t = q < 0 ? 0 : q / E + 1;       // lanes whose key > pos
                    const uint64_t msk = t >= 64 ? 0ull : (~0ull << t);
                    const uint64_t o = Om[e] & msk, c = Cm[e] & msk;
                    if (o) { const int kq = E * __builtin_ctzll(o) + e; if (kq < key) { key = kq; is_open = 1; } }
                    if (c) { const int kq = E * __builtin_ctzll(c) + e; if (kq < key) { key = kq; is_open = 0; } }
                }
                if (key == GATE_NOKEY) break;
                if (is_open) {
                    open_at(RL * k + key); seg_lo = key;
                } else {
                    seg(lane, k, nb, T, seg_lo, key, pm, pr, pi, m);
                    if (DEFER && OFS_GATE_DEFER) merge();
                    emit(lane, RL * k + key);
                    gate_open = 0; seg_lo = -1;
                }
                pos = key;
            }
        }
        if (gate_open) seg(lane, k, nb, T, seg_lo, RL - 1, pm, pr, pi, m);
    }

    // end of stream.  sync_aa: a gate still open closes at T (sync_aa.py:560-568);
    // minn_rtl: reported as open_gate_start (minn_rtl.py:814-823)
    __device__ __forceinline__ void finish(int lane, int T, int32_t* n_ev_out, int64_t* open_start = nullptr) {
        if constexpr (RTL) {
            if (lane == 0) {
                *n_ev_out = n_ev;
                if (open_start) *open_start = gate_open ? ev_start : -1;
            }
        } else {
            if (gate_open) { if (DEFER && OFS_GATE_DEFER) merge(); emit(lane, T); }
            if (lane == 0) *n_ev_out = n_ev;
        }
    }
};

}  // namespace ofs
