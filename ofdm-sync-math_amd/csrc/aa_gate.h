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
// RL·k + E·l + e.  Per row: prev-above by lane-serial + DPP max-scan, opens / closes by ballot,
// per-gate arg-extremum by wave max/min reductions; state carried between rows in scalars.
#pragma once
#include "ofs_common.h"

namespace ofs {

constexpr int GATE_NOKEY = 1 << 20;

template <int E, class V, bool RTL = false>
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
    }

    // the record is wave-uniform: lanes 0..3 store the four int64 fields and lanes 4..7 the four
    // f64 fields, one store instruction per 32-byte record half (a lane-0 loop of 8-byte stores
    // cost ~450 B of write traffic per event, measured with WRITE_SIZE)
    __device__ __forceinline__ void emit(int lane, int gate_end) {
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
        bool ab[E];
#pragma unroll
        for (int e = 0; e < E; ++e) ab[e] = (nb + e < T) && (double)m[e] >= thr;
        row_flags(lane, k, nb, T, ab, pm, pr, pi, m);
    }

    // generic row: above flags given; pm = the value whose arg-extremum is the peak
    __device__ __forceinline__ void row_flags(int lane, int k, int nb, int T, const bool (&ab)[E],
                                              const V (&pm)[E], const V (&pr)[E], const V (&pi)[E],
                                              const V (&m)[E]) {
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

        // arg-extremum of pm on keys [lo, hi]: sync_aa first max (strict >), minn_rtl last max (>=)
        auto seg_reduce = [&](int lo, int hi) {
            V lv = (V)-1, lpr = (V)0, lpi = (V)0, lm = (V)0;
            int lk = RTL ? -1 : GATE_NOKEY;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int key = E * lane + e;
                const bool in = nb + e < T && key >= lo && key <= hi;
                const bool better = RTL ? (pm[e] >= lv) : (pm[e] > lv);
                if (in && better) { lv = pm[e]; lk = key; lpr = pr[e]; lpi = pi[e]; lm = m[e]; }
            }
            const V vmax = wave_max(lv);
            const int kk = RTL ? wave_max_i(lv == vmax ? lk : -1) : wave_min(lv == vmax ? lk : GATE_NOKEY);
            const bool found = RTL ? (kk >= 0) : (kk != GATE_NOKEY);
            const bool take = RTL ? (vmax >= bpm) : (vmax > bpm);
            if (take && found) {
                const int ln = kk / E;
                bpr = readlane(lpr, ln);
                bpi = readlane(lpi, ln);
                bm = readlane(lm, ln);
                bpm = vmax;
                bidx = RL * k + kk;
            }
        };

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
                    gate_open = 1; ev_start = RL * k + key; seg_lo = key; bpm = (V)-1;
                } else {
                    seg_reduce(seg_lo, key);
                    emit(lane, RL * k + key);
                    gate_open = 0; seg_lo = -1;
                }
                pos = key;
            }
        }
        if (gate_open) seg_reduce(seg_lo, RL - 1);
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
            if (gate_open) emit(lane, T);
            if (lane == 0) *n_ev_out = n_ev;
        }
    }
};

}  // namespace ofs
