// ofdmsync.hip — MI355X (gfx950 / CDNA4) kernels + C ABI for the OFDM preamble-sync hot path.
//
// One engine covers every sliding-window timing metric of the reference:
// each is a window sum of a lagged product x[j]·conj(x[j-D]) plus a window sum of |x[j]|²,
// evaluated at a few prefix-sum offsets.  Per workgroup (256 threads = 4 wave64) and per
// stream tile:
//   A. coalesced loads of the tile (+ halo) into LDS, branch by branch; the lagged product
//      and the energy are formed from LDS and accumulated over branches;
//   B. prefix sums in fp64 (both precisions: an fp32 prefix difference cancels
//      catastrophically when a quiet window follows a loud burst): 4 samples per lane
//      serially, a wave64 inclusive scan per 256-sample row, row totals re-anchored;
//   C. outputs evaluated from prefix differences (lane-consecutive => fully coalesced stores);
//   D. (sync_aa detect) gate / peak / CFO events via a parallel formulation of the reference's
//      state machine (ballot bitmasks + LDS atomics), fused when the stream fits one tile.
// Hot path is HBM-bound (~1 flop/byte): no MFMA, see DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "ofdmsync.h"
#include "ofs_common.h"
#include <atomic>
#include <string.h>

namespace {

constexpr int WG = 256;            // threads per workgroup
constexpr int EPT = 4;             // scan elements per thread
constexpr int ROW = 64 * EPT;      // samples per wave-row (one fp64 re-anchor per row)
constexpr int PASS = WG * EPT;     // samples per scan pass
constexpr int EVBLK = 1024;        // positions per event-detection block
constexpr int MAXSLOT = 32;        // event slots per argmax round

enum Mode { M_AA = 0, M_SC = 1, M_COMB = 2, M_MINN = 3, M_RTL = 4 };

template <bool EX> struct Prec { using R = float; };
template <> struct Prec<true> { using R = double; };

template <int FMT, class R>
__device__ __forceinline__ void ldx(const void* p, int64_t i, R& re, R& im) {
    if constexpr (FMT == OFS_C64) {
        const float2 v = reinterpret_cast<const float2*>(p)[i];
        re = (R)v.x; im = (R)v.y;
    } else if constexpr (FMT == OFS_C128) {
        const double2 v = reinterpret_cast<const double2*>(p)[i];
        re = (R)v.x; im = (R)v.y;
    } else {
        const short2 v = reinterpret_cast<const short2*>(p)[i];
        re = (R)v.x; im = (R)v.y;
    }
}

template <class T>
__device__ __forceinline__ T wave_incl_scan(T s, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T t = __shfl_up(s, off, 64);
        if (lane >= off) s += t;
    }
    return s;
}

__device__ __forceinline__ double readlane_d(double v, int j) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), j);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), j);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ unsigned long long key_bits(float v) { return (unsigned long long)__float_as_uint(v); }
__device__ __forceinline__ unsigned long long key_bits(double v) { return (unsigned long long)__double_as_longlong(v); }

// ------------------------------------------------------------------------------------------
// Event detection for sync_aa (sync_aa.py:495-568), parallel over positions.
//
// Serial reference: gate opens on M >= thr; while open, peak = first argmax of |P|²
// (strict >); low_count counts consecutive M < thr, reset by an above sample; the gate
// closes at the sample where low_count reaches H' = max(H, 1); a gate still open at the end
// is closed at T.  Equivalent closed form used here, with prev(n) = last above position <= n:
//   close[n] <=> prev(n) exists and n - prev(n) == H'
//   open[n]  <=> above[n] and (prev(n-1) absent or (n-1) - prev(n-1) >= H')
// opens and closes alternate, so event k spans [open_k, close_k].  Positions < L are never
// valid (sync_aa.py:500-502), so the scan starts at L.
// ------------------------------------------------------------------------------------------
struct EvScratch {
    unsigned long long A[16], OB[16], CB[16];
    long long lastUpTo[16];
    int opfx[17], cpfx[17];
    unsigned long long slot_key[MAXSLOT];
    long long slot_idx[MAXSLOT];
    long long carry_last;     // last above position before the current block (-1: none)
    long long ev_start;
    unsigned long long best_key;
    long long best_idx;
    int open;                 // gate open entering the current block
    int open_at_start;
    int n_ev;
    int nslots;
};

// position of the k-th (0-based) set bit in words W[0..15]; -1 if absent
__device__ inline int select_bit(const unsigned long long* W, int k) {
    for (int w = 0; w < 16; ++w) {
        const int c = __popcll(W[w]);
        if (k < c) {
            unsigned long long m = W[w];
            for (int i = 0; i < k; ++i) m &= m - 1;
            return w * 64 + __ffsll((long long)m) - 1;
        }
        k -= c;
    }
    return -1;
}

template <class R, class GetMP, class GetP>
__device__ void aa_events(int64_t T, int L, double thr, int hyst, double fs, GetMP getmp,
                          GetP getp, int max_ev, int32_t* n_ev_out, int64_t* ev_i, double* ev_r,
                          EvScratch& s) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Hp = hyst > 1 ? hyst : 1;
    if (tid == 0) {
        s.carry_last = -1; s.open = 0; s.n_ev = 0; s.ev_start = 0; s.best_key = 0; s.best_idx = 0;
    }
    __syncthreads();

    auto emit = [&](long long gate_end) {   // thread 0 only
        const long long pk = s.best_idx;
        if (s.n_ev < max_ev) {
            double pr, pi;
            getp(pk, pr, pi);
            R m, pm;
            getmp(pk, m, pm);
            int64_t* ei = ev_i + (int64_t)s.n_ev * 4;
            double* er = ev_r + (int64_t)s.n_ev * 4;
            ei[0] = pk; ei[1] = s.ev_start; ei[2] = gate_end; ei[3] = pk - 2 * (long long)L + 1;
            er[0] = pr; er[1] = pi; er[2] = (double)m;
            er[3] = atan2(pi, pr) * fs / (2.0 * M_PI * (double)L);
        }
        s.n_ev += 1;
    };

    for (int64_t blk = L; blk < T; blk += EVBLK) {
        R mv[4], pmv[4];
        bool ab[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t n = blk + j * WG + tid;
            mv[j] = 0; pmv[j] = 0;
            if (n < T) getmp(n, mv[j], pmv[j]);
            ab[j] = (n < T) && ((double)mv[j] >= thr);
            const unsigned long long bal = __ballot(ab[j]);
            if (lane == 0) s.A[j * 4 + wave] = bal;
        }
        __syncthreads();
        if (tid == 0) {
            long long run = s.carry_last;
            for (int w = 0; w < 16; ++w) {
                if (s.A[w]) run = blk + w * 64 + 63 - __clzll((long long)s.A[w]);
                s.lastUpTo[w] = run;
            }
        }
        __syncthreads();
        bool opn[4], cls[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t n = blk + j * WG + tid;
            const int w = j * 4 + wave;
            const unsigned long long word = s.A[w];
            const long long before = (w > 0) ? s.lastUpTo[w - 1] : s.carry_last;
            const unsigned long long m_incl = (lane == 63) ? ~0ull : ((1ull << (lane + 1)) - 1);
            const unsigned long long m_excl = (1ull << lane) - 1;
            const unsigned long long wi = word & m_incl, we = word & m_excl;
            const long long base = blk + (long long)w * 64;
            const long long p_incl = wi ? base + 63 - __clzll((long long)wi) : before;
            const long long p_excl = we ? base + 63 - __clzll((long long)we) : before;
            const bool inb = n < T;
            cls[j] = inb && p_incl >= 0 && (n - p_incl) == Hp;
            opn[j] = inb && ab[j] && (p_excl < 0 || (n - 1 - p_excl) >= Hp);
            const unsigned long long bo = __ballot(opn[j]);
            const unsigned long long bc = __ballot(cls[j]);
            if (lane == 0) { s.OB[w] = bo; s.CB[w] = bc; }
        }
        __syncthreads();
        if (tid == 0) {
            s.opfx[0] = 0; s.cpfx[0] = 0;
            for (int w = 0; w < 16; ++w) {
                s.opfx[w + 1] = s.opfx[w] + __popcll(s.OB[w]);
                s.cpfx[w + 1] = s.cpfx[w] + __popcll(s.CB[w]);
            }
            s.open_at_start = s.open;
            s.nslots = s.opfx[16] + 1;    // slot 0 = carried gate (if any), slot k = k-th open
        }
        __syncthreads();
        // per position: slot and whether it is inside a gate
        int slot[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t n = blk + j * WG + tid;
            const int w = j * 4 + wave;
            const unsigned long long m_incl = (lane == 63) ? ~0ull : ((1ull << (lane + 1)) - 1);
            const unsigned long long m_excl = (1ull << lane) - 1;
            const int co = s.opfx[w] + __popcll(s.OB[w] & m_incl);   // opens <= n
            const int cc = s.cpfx[w] + __popcll(s.CB[w] & m_excl);   // closes < n
            const bool inside = (n < T) && (s.open_at_start + co - cc == 1);
            slot[j] = inside ? co : -1;
        }
        const int nslots = s.nslots;
        for (int r0 = 0; r0 < nslots; r0 += MAXSLOT) {
            if (tid < MAXSLOT) { s.slot_key[tid] = 0; s.slot_idx[tid] = 0x7fffffffffffffffll; }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (slot[j] >= r0 && slot[j] < r0 + MAXSLOT)
                    atomicMax(&s.slot_key[slot[j] - r0], key_bits(pmv[j]));
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (slot[j] >= r0 && slot[j] < r0 + MAXSLOT &&
                    key_bits(pmv[j]) == s.slot_key[slot[j] - r0])
                    atomicMin(&s.slot_idx[slot[j] - r0], (long long)(blk + j * WG + tid));
            __syncthreads();
            if (tid == 0) {
                const int rend = min(nslots, r0 + MAXSLOT);
                for (int k = r0; k < rend; ++k) {
                    if (k == 0 && !s.open_at_start) continue;    // no carried gate
                    const unsigned long long key = s.slot_key[k - r0];
                    const long long idx = s.slot_idx[k - r0];
                    if (k == 0) {
                        if (idx != 0x7fffffffffffffffll && key > s.best_key) { s.best_key = key; s.best_idx = idx; }
                    } else {
                        s.ev_start = blk + select_bit(s.OB, k - 1);
                        s.best_key = key; s.best_idx = idx;
                    }
                    // which close ends this gate
                    const int ci = s.open_at_start ? k : k - 1;
                    if (ci < s.cpfx[16]) {
                        emit(blk + select_bit(s.CB, ci));
                        s.open = 0;
                    } else {
                        s.open = 1;
                    }
                }
            }
            __syncthreads();
        }
        if (tid == 0) s.carry_last = s.lastUpTo[15];
        __syncthreads();
    }
    if (tid == 0) {
        if (s.open) emit(T);
        *n_ev_out = s.n_ev;
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------
// Window-metric engine
// ------------------------------------------------------------------------------------------
struct WinArgs {
    const void* x;
    int64_t T, n_out, chunk;
    int32_t nb, n_chunks;
    int32_t D, W, N, Q;
    int32_t lo_x, hi_x;
    int32_t len_max, nrows_max;
    void* P; void* R; void* M; uint8_t* valid;
    double* corr_total; double* corr_positive; double* energy_total; double* energy_scaled;
    uint8_t* mvalid;
    double thr_value;
    int32_t detect; double thr; int32_t hyst; double fs; int32_t max_ev;
    int32_t* n_ev; int64_t* ev_i; double* ev_r;
};

template <int MODE> struct NQ { static constexpr int v = 3; };
template <> struct NQ<M_RTL> { static constexpr int v = 2; };

template <class R>
__host__ __device__ constexpr size_t win_lds_bytes(int len_max, int nrows_max, int nq) {
    return (size_t)len_max * 2 * sizeof(R) + (size_t)nq * len_max * sizeof(double) +
           (size_t)nq * nrows_max * sizeof(double) + sizeof(EvScratch) + 64;
}

template <int FMT, bool EX, int MODE>
__global__ __launch_bounds__(WG) void win_kernel(WinArgs a) {
    using R = typename Prec<EX>::R;
    constexpr int NQV = NQ<MODE>::v;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t b = blockIdx.x / a.n_chunks;
    const int64_t c = blockIdx.x % a.n_chunks;
    const int64_t c0 = c * a.chunk;
    const int64_t c1 = min(c0 + a.chunk, a.n_out);
    const int64_t ls = max((int64_t)0, c0 + a.lo_x);
    const int64_t le = min(a.T, c1 - 1 + a.hi_x + 1);
    const int len = (int)(le - ls);
    const int LM = a.len_max, NRM = a.nrows_max;

    R* xs = reinterpret_cast<R*>(smem);                       // [LM][2]
    double* acc = reinterpret_cast<double*>(xs + 2 * LM);     // [NQV][LM] (fp64 prefix)
    double* rows = reinterpret_cast<double*>(acc + NQV * LM); // [NQV][NRM]
    EvScratch* evs = reinterpret_cast<EvScratch*>(rows + NQV * NRM);

    // ---- A: branch loop, lagged product + energy accumulated over branches ----
    for (int br = 0; br < a.nb; ++br) {
        const int64_t base = (b * a.nb + br) * a.T + ls;
        for (int i = tid; i < len; i += WG) {
            R re, im;
            ldx<FMT, R>(a.x, base + i, re, im);
            xs[2 * i] = re; xs[2 * i + 1] = im;
        }
        __syncthreads();
        for (int i = tid; i < len; i += WG) {
            // products in fp64 from the stored samples (exact for fp32 / int16 samples)
            const double re = xs[2 * i], im = xs[2 * i + 1];
            const double e = re * re + im * im;
            double pr = 0, pi = 0;
            if (i >= a.D) {
                const double dr = xs[2 * (i - a.D)], di = xs[2 * (i - a.D) + 1];
                if constexpr (MODE == M_RTL) {
                    pr = dr * re + di * im;          // minn_rtl.py:616
                } else {
                    pr = re * dr + im * di;          // x[j]·conj(x[j-D])
                    pi = im * dr - re * di;
                }
            }
            if (br == 0) {
                acc[i] = pr;
                if constexpr (NQV == 3) acc[LM + i] = pi;
                acc[(NQV - 1) * LM + i] = e;
            } else {
                acc[i] += pr;
                if constexpr (NQV == 3) acc[LM + i] += pi;
                acc[(NQV - 1) * LM + i] += e;
            }
        }
        __syncthreads();
    }

    // ---- B: prefix sums (in place) + fp64 row re-anchoring ----
    for (int p0 = 0; p0 < len; p0 += PASS) {
        const int i0 = p0 + tid * EPT;
#pragma unroll
        for (int q = 0; q < NQV; ++q) {
            double v[EPT];
#pragma unroll
            for (int k = 0; k < EPT; ++k) v[k] = (i0 + k < len) ? acc[q * LM + i0 + k] : 0.0;
#pragma unroll
            for (int k = 1; k < EPT; ++k) v[k] += v[k - 1];
            const double incl = wave_incl_scan(v[EPT - 1], lane);
            double excl = __shfl_up(incl, 1, 64);
            if (lane == 0) excl = 0;
#pragma unroll
            for (int k = 0; k < EPT; ++k)
                if (i0 + k < len) acc[q * LM + i0 + k] = v[k] + excl;
            if (lane == 63) rows[q * NRM + p0 / ROW + wave] = (double)incl;
        }
    }
    __syncthreads();
    if (tid < NQV) {
        const int nrows = (len + ROW - 1) / ROW;
        double run = 0.0;
        for (int r = 0; r < nrows; ++r) {
            const double t = rows[tid * NRM + r];
            rows[tid * NRM + r] = run;
            run += t;
        }
    }
    __syncthreads();

    auto pref = [&](int q, int64_t li) -> double {
        if (li < 0) return 0.0;
        return rows[q * NRM + (int)(li / ROW)] + acc[q * LM + li];
    };

    // ---- C: outputs ----
    const bool fused_detect = (MODE == M_AA) && a.detect && a.n_chunks == 1;
    R* ml = xs;                // aliases xs (free after A): M and |P|² per local position
    R* pml = xs + LM;
    for (int64_t o = c0 + tid; o < c1; o += WG) {
        const int64_t oi = b * a.n_out + o;
        if constexpr (MODE == M_RTL) {
            const int Q = a.Q;
            const int64_t i = o;
            auto C = [&](int64_t g) { return pref(0, g - ls) - pref(0, g - Q - ls); };
            auto E = [&](int64_t g) { return pref(1, g - ls) - pref(1, g - Q - ls); };
            double ct = (i >= Q - 1 ? C(i) : 0.0);
            ct = ct + (i >= 2 * Q - 1 ? C(i - Q) : 0.0);
            double et = (i >= Q - 1 ? E(i) : 0.0);
            et = et + (i >= 2 * Q - 1 ? E(i - Q) : 0.0);
            et = et + (i >= 3 * Q - 1 ? E(i - 2 * Q) : 0.0);
            a.corr_total[oi] = ct;
            if (a.corr_positive) a.corr_positive[oi] = ct > 0.0 ? ct : 0.0;
            a.energy_total[oi] = et;
            if (a.energy_scaled) a.energy_scaled[oi] = (a.thr_value == 0.0) ? 0.0 : et * a.thr_value;
            if (a.mvalid) a.mvalid[oi] = (i >= 3 * (int64_t)Q - 1);
        } else {
            double Pr, Pi, Rr;
            bool ok;
            if constexpr (MODE == M_AA) {
                const int64_t li = o - ls, L = a.W;
                Pr = pref(0, li) - pref(0, li - L);
                Pi = pref(1, li) - pref(1, li - L);
                Rr = pref(2, li) - pref(2, li - L);
                ok = o >= L;
            } else if constexpr (MODE == M_SC || MODE == M_COMB) {
                const int64_t half = a.W, N = a.N;
                const int64_t le_ = o + N - 1 - ls, lm_ = o + half - 1 - ls;
                Pr = pref(0, le_) - pref(0, lm_);
                Pi = -(pref(1, le_) - pref(1, lm_));
                Rr = pref(2, le_) - pref(2, (MODE == M_COMB ? o - 1 : o + half - 1) - ls);
                ok = true;
            } else {  // M_MINN
                const int64_t Q = a.Q;
                const int64_t a1 = o + 2 * Q - 1 - ls, a0 = o + Q - 1 - ls;
                const int64_t b1 = o + 4 * Q - 1 - ls, b0 = o + 3 * Q - 1 - ls;
                Pr = (pref(0, a1) - pref(0, a0)) + (pref(0, b1) - pref(0, b0));
                Pi = -((pref(1, a1) - pref(1, a0)) + (pref(1, b1) - pref(1, b0)));
                Rr = pref(2, b1) - pref(2, a0);
                ok = true;
            }
            // metric in fp64 (sync_aa.py:486-493, sc.py:76-77, minn.py:109-111), stored as R
            const R pr = (R)Pr, pi = (R)Pi, rr = (R)Rr;
            const double pmd = Pr * Pr + Pi * Pi;
            double md;
            if constexpr (MODE == M_AA) {
                md = (ok && Rr > 1e-6 * (double)a.W) ? pmd / (Rr * Rr) : 0.0;
                md = md < 1.0 ? md : 1.0;
            } else if constexpr (MODE == M_MINN) {
                const double re_pos = Pr > 0.0 ? Pr : 0.0;
                const double den = Rr > 1e-12 ? Rr : 1e-12;
                md = re_pos * re_pos / (den * den);
            } else {
                const double den = Rr > 1e-12 ? Rr : 1e-12;
                md = pmd / (den * den);
            }
            const R m = (R)md, pm = (R)pmd;
            if (a.P) { R* P = reinterpret_cast<R*>(a.P); P[2 * oi] = pr; P[2 * oi + 1] = pi; }
            if (a.R) reinterpret_cast<R*>(a.R)[oi] = rr;
            if (a.M) reinterpret_cast<R*>(a.M)[oi] = m;
            if constexpr (MODE == M_AA) {
                if (a.valid) a.valid[oi] = ok;
                if (fused_detect) { ml[o - ls] = m; pml[o - ls] = pm; }
            }
        }
    }

    // ---- D: fused event detection (whole stream in this tile) ----
    if constexpr (MODE == M_AA) {
        if (fused_detect) {
            __syncthreads();
            const int L = a.W;
            auto getmp = [&](int64_t n, R& m, R& pm) { m = ml[n]; pm = pml[n]; };
            auto getp = [&](int64_t n, double& pr, double& pi) {
                pr = (double)(R)(pref(0, n) - pref(0, n - L));
                pi = (double)(R)(pref(1, n) - pref(1, n - L));
            };
            aa_events<R>(a.T, L, a.thr, a.hyst, a.fs, getmp, getp, a.max_ev, a.n_ev + b,
                         a.ev_i + b * (int64_t)a.max_ev * 4, a.ev_r + b * (int64_t)a.max_ev * 4, *evs);
        }
    }
    (void)lane; (void)wave;
}

// Event detection over P/M already in global memory (streams longer than one tile).
template <bool EX>
__global__ __launch_bounds__(WG) void aa_events_kernel(const void* Pg, const void* Mg, int64_t T,
                                                      int L, double thr, int hyst, double fs,
                                                      int max_ev, int32_t* n_ev, int64_t* ev_i,
                                                      double* ev_r) {
    using R = typename Prec<EX>::R;
    __shared__ EvScratch evs;
    const int64_t b = blockIdx.x;
    const R* P = reinterpret_cast<const R*>(Pg) + 2 * b * T;
    const R* M = reinterpret_cast<const R*>(Mg) + b * T;
    auto getmp = [&](int64_t n, R& m, R& pm) {
        m = M[n];
        const R pr = P[2 * n], pi = P[2 * n + 1];
        pm = pr * pr + pi * pi;
    };
    auto getp = [&](int64_t n, double& pr, double& pi) { pr = P[2 * n]; pi = P[2 * n + 1]; };
    aa_events<R>(T, L, thr, hyst, fs, getmp, getp, max_ev, n_ev + b, ev_i + b * (int64_t)max_ev * 4,
                 ev_r + b * (int64_t)max_ev * 4, evs);
}

// ------------------------------------------------------------------------------------------
// minn_rtl: sequential IIR smoothing + threshold + gate FSM (minn_rtl.py:704-722, :750-825).
// One wave per stream; values are broadcast lane by lane (readlane) so the recursion is the
// exact float64 operation sequence of the reference.
// ------------------------------------------------------------------------------------------
struct RtlArgs {
    const double* corr_total; const double* energy_total;
    double* smooth; double* corr_scaled; uint8_t* above;
    int64_t T; int32_t Q, shift, smooth_mode, frac_bits; double thr_value;
    int32_t detect, hyst, toff, max_ev; int32_t* n_ev; int64_t* ev; int64_t* open_start;
};

// Lane-per-stream form: wave 0 of a 256-thread workgroup is the WORKER — one lane per stream,
// 64 streams — and walks its stream's samples sequentially (recursion, threshold compare and
// gate FSM are per-lane scalar code, no idle lanes).  Waves 1-3 are LOADERS: they stage chunk
// c+1 of the 64 streams from HBM into an LDS ring (coalesced rows: a row is one stream's RCH
// consecutive samples) and write chunk c-1's results back while the worker runs chunk c; one
// barrier per chunk.  With only B/64 workgroups in flight the loaders are what keeps the
// memory system busy.
constexpr int RCH = 64;
constexpr int RNB = 2;                                   // LDS ring depth: loaders store c-1 then refill it with c+1

struct RtlRing {
    double c[RNB][64][RCH + 1];                          // corr_positive in, smooth out
    double e[RNB][64][RCH + 1];                          // energy_scaled in, corr_scaled out
    uint8_t f[RNB][64][RCH + 4];                         // above out
};

__global__ __launch_bounds__(256) void rtl_iir_kernel(RtlArgs a, int64_t B) {
#pragma clang fp contract(off)
    __shared__ RtlRing ring;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int64_t b0 = (int64_t)blockIdx.x * 64;
    const int nst = (int)min((int64_t)64, B - b0);         // streams of this workgroup
    const int64_t T = a.T;
    const int nch = (int)((T + RCH - 1) / RCH);
    const int64_t vstart = 3 * (int64_t)a.Q - 1;
    const double inv = ldexp(1.0, -(a.shift > 0 ? a.shift : 0));   // exact 1 / 2^shift
    const double scale = (double)(1ll << a.frac_bits);

    // loader helpers (waves 1-3: 192 threads sweep the 64 x RCH tile)
    const int lt = tid - 64;
    auto load_chunk = [&](int c) {
        const int64_t base = (int64_t)c * RCH;
        const int cnt = (int)min((int64_t)RCH, T - base);
        const int buf = c % RNB;
        constexpr int PER_T = (64 * RCH + 191) / 192;
        double vc[PER_T], ve[PER_T];
#pragma unroll
        for (int i = 0; i < PER_T; ++i) {
            const int el = lt + 192 * i, r = el / RCH, col = el % RCH;
            const bool ok = el < 64 * RCH && r < nst && col < cnt;
            const int64_t g = (b0 + r) * T + base + col;
            vc[i] = ok ? a.corr_total[g] : 0.0;
            ve[i] = ok ? a.energy_total[g] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < PER_T; ++i) {
            const int el = lt + 192 * i, r = el / RCH, col = el % RCH;
            if (el < 64 * RCH) {
                ring.c[buf][r][col] = vc[i] > 0.0 ? vc[i] : 0.0;
                ring.e[buf][r][col] = (a.thr_value == 0.0) ? 0.0 : ve[i] * a.thr_value;
            }
        }
    };
    auto store_chunk = [&](int c) {
        const int64_t base = (int64_t)c * RCH;
        const int cnt = (int)min((int64_t)RCH, T - base);
        const int buf = c % RNB;
        for (int el = lt; el < 64 * RCH; el += 192) {
            const int r = el / RCH, col = el % RCH;
            if (r < nst && col < cnt) {
                const int64_t g = (b0 + r) * T + base + col;
                if (a.smooth) a.smooth[g] = ring.c[buf][r][col];
                if (a.corr_scaled) a.corr_scaled[g] = ring.e[buf][r][col];
                if (a.above) a.above[g] = ring.f[buf][r][col];
            }
        }
    };

    // worker state (wave 0, lane = stream)
    const int64_t b = b0 + lane;
    double sm = 0.0;
    long long si = 0;
    bool gate_open = false;
    long long gate_start = -1, peak_index = 0;
    double peak_value = 0.0;
    int low = 0, n_ev = 0;
    const int hyst_limit = a.hyst > 0 ? a.hyst - 1 : 0;
    int64_t* ev = (wave == 0 && a.ev && b < B) ? a.ev + b * (int64_t)a.max_ev * 4 : nullptr;

    if (wave > 0) load_chunk(0);
    __syncthreads();
    for (int c = 0; c <= nch; ++c) {
        if (wave == 0) {
            if (c < nch && lane < nst) {
                const int buf = c % RNB;
                const int64_t base = (int64_t)c * RCH;
                const int cnt = (int)min((int64_t)RCH, T - base);
#pragma unroll 4
                for (int j = 0; j < cnt; ++j) {
                    const int64_t idx = base + j;
                    const double cpj = ring.c[buf][lane][j];
                    const double esj = ring.e[buf][lane][j];
                    const bool vj = idx >= vstart;
                    if (vj) {
                        if (a.smooth_mode == 0) {
                            if (a.shift == 0) sm = cpj;
                            else sm = sm + (cpj - sm) * inv;
                        } else {
                            const long long ci = (long long)cpj;
                            si = (a.shift == 0) ? ci : si + ((ci - si) >> a.shift);
                            sm = (double)si;
                        }
                    }
                    const double cs = sm * scale;
                    const bool abv = vj && (cs >= esj);
                    ring.c[buf][lane][j] = sm;
                    ring.e[buf][lane][j] = cs;
                    ring.f[buf][lane][j] = (uint8_t)abv;
                    if (a.detect && vj) {
                        if (!gate_open) {
                            if (abv) { gate_open = true; gate_start = idx; peak_value = cpj; peak_index = idx; low = 0; }
                        } else {
                            if (cpj >= peak_value) { peak_value = cpj; peak_index = idx; }
                            if (abv) {
                                low = 0;
                            } else {
                                const bool closing = (a.hyst == 0) || (low == hyst_limit);
                                if (!closing) low += 1;
                                if (closing) {
                                    if (ev && n_ev < a.max_ev) {
                                        int64_t* rr = ev + (int64_t)n_ev * 4;
                                        rr[0] = peak_index; rr[1] = peak_index + a.toff; rr[2] = gate_start; rr[3] = idx + 1;
                                    }
                                    n_ev += 1;
                                    gate_open = false; gate_start = -1; peak_value = 0.0; low = 0;
                                }
                            }
                        }
                    }
                }
            }
        } else {
            if (c >= 1) store_chunk(c - 1);
            if (c + 1 < nch) load_chunk(c + 1);
        }
        __syncthreads();
    }
    if (wave == 0 && a.detect && b < B) {
        a.n_ev[b] = n_ev;
        if (a.open_start) a.open_start[b] = gate_open ? gate_start : -1;
    }
}

// Gate FSM alone on precomputed arrays (detect_minn_rtl on an existing state).
__global__ __launch_bounds__(64) void rtl_gate_kernel(const double* cpos, const uint8_t* above,
                                                     const uint8_t* valid, int64_t T, int hyst,
                                                     int toff, int max_ev, int32_t* n_ev_out,
                                                     int64_t* ev_all, int64_t* open_start) {
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    bool gate_open = false;
    long long gate_start = -1, peak_index = 0;
    double peak_value = 0.0;
    int low = 0, n_ev = 0;
    const int hyst_limit = hyst > 0 ? hyst - 1 : 0;
    int64_t* ev = ev_all ? ev_all + b * (int64_t)max_ev * 4 : nullptr;
    for (int64_t base = 0; base < T; base += 64) {
        const int64_t n = base + lane;
        const bool inb = n < T;
        const double cp = inb ? cpos[b * T + n] : 0.0;
        const int ab = inb ? (int)above[b * T + n] : 0;
        const int vd = inb ? (int)valid[b * T + n] : 0;
        const unsigned long long abm = __ballot(ab != 0);
        const unsigned long long vdm = __ballot(vd != 0);
        const int jend = (int)min((int64_t)64, T - base);
        for (int j = 0; j < jend; ++j) {
            if (!((vdm >> j) & 1ull)) continue;
            const int64_t idx = base + j;
            const double cpj = readlane_d(cp, j);
            const bool abv = (abm >> j) & 1ull;
            if (!gate_open) {
                if (abv) { gate_open = true; gate_start = idx; peak_value = cpj; peak_index = idx; low = 0; }
            } else {
                if (cpj >= peak_value) { peak_value = cpj; peak_index = idx; }
                if (abv) {
                    low = 0;
                } else {
                    const bool closing = (hyst == 0) || (low == hyst_limit);
                    if (!closing) low += 1;
                    if (closing) {
                        if (lane == 0 && n_ev < max_ev) {
                            int64_t* r = ev + (int64_t)n_ev * 4;
                            r[0] = peak_index; r[1] = peak_index + toff; r[2] = gate_start; r[3] = idx + 1;
                        }
                        n_ev += 1;
                        gate_open = false; gate_start = -1; peak_value = 0.0; low = 0;
                    }
                }
            }
        }
    }
    if (lane == 0) {
        n_ev_out[b] = n_ev;
        if (open_start) open_start[b] = gate_open ? gate_start : -1;
    }
}

// ------------------------------------------------------------------------------------------
// CP-correlation CFO (core.py:179-196): one workgroup per stream, fp64 reduction.
// ------------------------------------------------------------------------------------------
template <int FMT>
__global__ __launch_bounds__(WG) void cp_cfo_kernel(const void* x, int64_t T, int nb,
                                                   const int64_t* starts, int n_fft, int cp_len,
                                                   double fs, double* P_out, double* cfo_out) {
    __shared__ double red[2][WG / 64];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t st = starts[b];
    double pr = 0.0, pi = 0.0;
    for (int br = 0; br < nb; ++br) {
        const int64_t base = (b * nb + br) * T;
        for (int k = tid; k < cp_len; k += WG) {
            double ar, ai, br_, bi;
            ldx<FMT, double>(x, base + st + k, ar, ai);
            ldx<FMT, double>(x, base + st + n_fft + k, br_, bi);
            pr += ar * br_ + ai * bi;          // a * conj(b)
            pi += ai * br_ - ar * bi;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        pr += __shfl_xor(pr, off, 64);
        pi += __shfl_xor(pi, off, 64);
    }
    if (lane == 0) { red[0][wave] = pr; red[1][wave] = pi; }
    __syncthreads();
    if (tid == 0) {
        double sr = 0.0, si = 0.0;
        for (int w = 0; w < WG / 64; ++w) { sr += red[0][w]; si += red[1][w]; }
        if (P_out) { P_out[2 * b] = sr; P_out[2 * b + 1] = si; }
        cfo_out[b] = -atan2(si, sr) * fs / (2.0 * M_PI * (double)n_fft);
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
constexpr int LEN_MAX_FP32 = 3072;   // 32 B/sample of LDS  -> 96 KiB tiles
constexpr int LEN_MAX_FP64 = 3584;   // 40 B/sample of LDS  -> 140 KiB tiles

struct Plan { int64_t chunk; int32_t n_chunks, len_max, nrows_max; size_t lds; };

template <class R>
static int make_plan(int64_t T, int64_t n_out, int lo_x, int hi_x, int nq, bool exact, Plan& p) {
    const int halo = hi_x - lo_x;
    const int len_cap = exact ? LEN_MAX_FP64 : LEN_MAX_FP32;
    const int64_t chunk_cap = (int64_t)len_cap - halo;
    if (chunk_cap < 1) return OFS_ETOOLONG;
    int64_t n_chunks = (n_out + chunk_cap - 1) / chunk_cap;
    if (n_chunks < 1) n_chunks = 1;
    int64_t chunk = (n_out + n_chunks - 1) / n_chunks;
    int64_t max_len = chunk + halo;
    if (max_len > T) max_len = T;
    int len_max = (int)((max_len + 3) & ~3ll);
    if (len_max < 4) len_max = 4;
    const int nrows_max = ((len_max + PASS - 1) / PASS) * (PASS / ROW);
    p.chunk = chunk; p.n_chunks = (int32_t)n_chunks; p.len_max = len_max; p.nrows_max = nrows_max;
    p.lds = win_lds_bytes<R>(len_max, nrows_max, nq);
    return OFS_OK;
}

template <int FMT, bool EX, int MODE>
static int launch_win(WinArgs a, int64_t B, const Plan& p, hipStream_t st) {
    auto k = win_kernel<FMT, EX, MODE>;
    if (p.lds > 65536) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds) != hipSuccess)
            return OFS_EHIP;
    }
    a.chunk = p.chunk; a.n_chunks = p.n_chunks; a.len_max = p.len_max; a.nrows_max = p.nrows_max;
    const int64_t grid = B * (int64_t)p.n_chunks;
    if (grid > 0x7fffffffll) return OFS_EINVAL;
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(WG), p.lds, st, a);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

template <int MODE>
static int dispatch_win(int fmt, int precision, WinArgs a, int64_t B, int lo_x, int hi_x,
                        hipStream_t st, Plan* plan_out) {
    constexpr int nq = NQ<MODE>::v;
    Plan p;
    int rc;
    const bool ex = precision == OFS_FP64;
    rc = ex ? make_plan<double>(a.T, a.n_out, lo_x, hi_x, nq, true, p)
            : make_plan<float>(a.T, a.n_out, lo_x, hi_x, nq, false, p);
    if (rc) return rc;
    if (plan_out) *plan_out = p;
    a.lo_x = lo_x; a.hi_x = hi_x;
    if (ex) {
        switch (fmt) {
            case OFS_C64: return launch_win<OFS_C64, true, MODE>(a, B, p, st);
            case OFS_C128: return launch_win<OFS_C128, true, MODE>(a, B, p, st);
            case OFS_CI16: return launch_win<OFS_CI16, true, MODE>(a, B, p, st);
        }
    } else if constexpr (MODE != M_RTL) {
        switch (fmt) {
            case OFS_C64: return launch_win<OFS_C64, false, MODE>(a, B, p, st);
            case OFS_C128: return launch_win<OFS_C128, false, MODE>(a, B, p, st);
            case OFS_CI16: return launch_win<OFS_CI16, false, MODE>(a, B, p, st);
        }
    }
    return OFS_EINVAL;
}

static bool fmt_ok(int f) { return f == OFS_C64 || f == OFS_C128 || f == OFS_CI16; }
static bool prec_ok(int p) { return p == OFS_FP32 || p == OFS_FP64; }

}  // namespace

// ==========================================================================================
// C ABI
// ==========================================================================================
extern "C" {

int32_t ofs_version(void) { return 100; }

// ofs_source_hash / ofs_source_tag (the hash of the sources this binary was compiled from) live
// in a one-line translation unit __graft_entry__.build_hip generates, so a source edit does not
// force this file to recompile.

static const char* const kVariantNames[ofs::V_COUNT] = {
    "EXACT", "FAST_E", "FAST_E_DO", "FAST_SCAN", "FAST_SCAN_DO", "RTL_WPB", "PARK_DIRECT", "ZW64",
    "ZW64_GRID", "ZS", "ZF_ITEMS", "ZS_PAIR", "ZS_DEFER", "ZS_BPL", "ZS_C", "ZS_GBLK", "MC_FUSED",
    "MC_FUSE_X", "ZC_SEQ", "ZC_NODMA", "BE_FAST", "MC_PERS", "FAST_LDS", "OCC_LDS"};
// Per calling thread: a variant one thread sets steers only the calls that thread makes, so
// concurrent callers (another thread's production calls) never see a test's forced kernel.
struct VariantTable {
    int64_t v[ofs::V_COUNT];
    VariantTable() { for (auto& x : v) x = OFS_VARIANT_UNSET; }
};
static thread_local VariantTable g_variants;

static int variant_index(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < ofs::V_COUNT; ++i)
        if (strcmp(name, kVariantNames[i]) == 0) return i;
    return -1;
}

int32_t ofs_debug_reset_variants(void) {
    for (auto& x : g_variants.v) x = OFS_VARIANT_UNSET;
    return OFS_OK;
}

int32_t ofs_debug_set_variant(const char* name, int64_t value) {
    const int i = variant_index(name);
    if (i < 0) return OFS_EINVAL;
    g_variants.v[i] = value;
    return OFS_OK;
}

int64_t ofs_debug_get_variant(const char* name) {
    const int i = variant_index(name);
    return i < 0 ? OFS_VARIANT_UNSET : ofs::variant((ofs::Variant)i);
}

const char* ofs_status_string(int32_t s) {
    switch (s) {
        case OFS_OK: return "ok";
        case OFS_EINVAL: return "invalid argument";
        case OFS_ETOOLONG: return "window/halo does not fit one LDS tile";
        case OFS_EHIP: return "HIP launch error";
        case OFS_ESHORT: return "stream shorter than one symbol";
        case OFS_EFFT: return "rocFFT error";
        default: return "unknown status";
    }
}

int32_t ofs_aa_detect(int32_t in_fmt, const void* x, int64_t B, int32_t n_ant, int64_t T,
                      int32_t L, int32_t precision, void* P, void* R, void* M, uint8_t* valid,
                      int32_t detect, double threshold, int32_t hysteresis, double sample_rate,
                      int32_t max_events, int32_t* n_events, int64_t* ev_int, double* ev_real,
                      void* stream) {
    if (!(fmt_ok(in_fmt) || in_fmt == OFS_CP12) || !prec_ok(precision) || OFS_MISSING(x, B * T) || B < 0 || n_ant < 1 ||
        T < 0 || L < 1)
        return OFS_EINVAL;
    if (detect && (OFS_MISSING(n_events, B) || max_events < 0 ||
                   (max_events > 0 && B > 0 && (!ev_int || !ev_real))))
        return OFS_EINVAL;
    if (B == 0 || T == 0) return OFS_OK;
    hipStream_t st = (hipStream_t)stream;
    {   // register-resident fast path (aa_fast.hip) when the shape allows it
        AaFastArgs f{};
        f.x = x; f.B = B; f.T = T; f.L = L; f.P = P; f.R = R; f.M = M; f.valid = valid;
        f.detect = detect; f.thr = threshold; f.hyst = hysteresis; f.fs = sample_rate;
        f.max_ev = max_events; f.n_ev = n_events; f.ev_i = ev_int; f.ev_r = ev_real;
        int frc = ofs_aa_fast_try(in_fmt, precision, n_ant, f, st);
        if (frc == 1) return OFS_OK;
        if (frc < 0) return frc;
        frc = ofs_aa_exact_try(in_fmt, precision, n_ant, f, st);      // int16 I/Q, fp64 (aa_exact.hip)
        if (frc == 1) return OFS_OK;
        if (frc < 0) return frc;
    }
    if (in_fmt == OFS_CP12) return OFS_EINVAL;                        // packed words: exact kernels only
    WinArgs a{};
    a.x = x; a.T = T; a.n_out = T; a.nb = n_ant; a.D = L; a.W = L;
    a.P = P; a.R = R; a.M = M; a.valid = valid;
    a.detect = detect; a.thr = threshold; a.hyst = hysteresis; a.fs = sample_rate;
    a.max_ev = max_events; a.n_ev = n_events; a.ev_i = ev_int; a.ev_r = ev_real;
    const int lo = -(int)(2 * (int64_t)L - 1);
    if (2 * (int64_t)L - 1 > 0x3fffffff) return OFS_ETOOLONG;
    Plan p;
    // decide fusion before launching: detect on a multi-tile stream needs P and M in HBM
    {
        Plan probe;
        const bool ex = precision == OFS_FP64;
        const int rc = ex ? make_plan<double>(T, T, lo, 0, 3, true, probe)
                          : make_plan<float>(T, T, lo, 0, 3, false, probe);
        if (rc) return rc;
        if (detect && probe.n_chunks > 1 && (!P || !M)) return OFS_EINVAL;
    }
    int rc = dispatch_win<M_AA>(in_fmt, precision, a, B, lo, 0, st, &p);
    if (rc) return rc;
    if (detect && p.n_chunks > 1) {
        if (precision == OFS_FP64)
            hipLaunchKernelGGL(aa_events_kernel<true>, dim3((unsigned)B), dim3(WG), 0, st, P, M, T, L,
                               threshold, hysteresis, sample_rate, max_events, n_events, ev_int, ev_real);
        else
            hipLaunchKernelGGL(aa_events_kernel<false>, dim3((unsigned)B), dim3(WG), 0, st, P, M, T, L,
                               threshold, hysteresis, sample_rate, max_events, n_events, ev_int, ev_real);
        if (hipGetLastError() != hipSuccess) return OFS_EHIP;
    }
    return OFS_OK;
}

int32_t ofs_aa_plan(int32_t in_fmt, int32_t precision, int32_t n_ant, int64_t T, int32_t L) {
    if (!(fmt_ok(in_fmt) || in_fmt == OFS_CP12) || !prec_ok(precision) || n_ant < 1 || T < 0 || L < 1) return OFS_EINVAL;
    const int fp = ofs_aa_fast_plan(in_fmt, precision, n_ant, T, L);
    if (fp) return 1000 + fp;
    const int xp = ofs_aa_exact_plan(in_fmt, precision, n_ant, T, L);
    if (xp) return (xp >= 100 ? 3000 : 2000) + xp % 100;
    if (in_fmt == OFS_CP12) return OFS_EINVAL;
    if (2 * (int64_t)L - 1 > 0x3fffffff) return OFS_ETOOLONG;
    Plan p;
    const int lo = -(int)(2 * (int64_t)L - 1);
    const int rc = precision == OFS_FP64 ? make_plan<double>(T > 0 ? T : 1, T > 0 ? T : 1, lo, 0, 3, true, p)
                                         : make_plan<float>(T > 0 ? T : 1, T > 0 ? T : 1, lo, 0, 3, false, p);
    if (rc) return rc;
    return p.n_chunks > 1 ? 2 : 1;
}

int32_t ofs_sc_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                      int32_t symbol_len, int32_t r_mode, int32_t precision,
                      void* M, void* P, void* R, void* stream) {
    if (!fmt_ok(in_fmt) || !prec_ok(precision) || OFS_MISSING(x, B * T) || B < 0 || n_br < 1 || T < 0)
        return OFS_EINVAL;
    if (symbol_len < 2 || (symbol_len & 1) || (r_mode != 0 && r_mode != 1)) return OFS_EINVAL;
    const int64_t n_out = T - symbol_len + 1;
    if (B == 0 || n_out <= 0) return OFS_OK;
    hipStream_t st = (hipStream_t)stream;
    {
        const WinFastArgs f{x, B, T, symbol_len, M, P, R};
        const int frc = ofs_win_fast_try(r_mode == 0 ? 1 : 2, in_fmt, precision, n_br, f, st);
        if (frc != 0) return frc > 0 ? OFS_OK : frc;
    }
    WinArgs a{};
    a.x = x; a.T = T; a.n_out = n_out; a.nb = n_br; a.D = symbol_len / 2; a.W = symbol_len / 2;
    a.N = symbol_len; a.P = P; a.R = R; a.M = M;
    return r_mode == 0 ? dispatch_win<M_SC>(in_fmt, precision, a, B, 0, symbol_len - 1, st, nullptr)
                       : dispatch_win<M_COMB>(in_fmt, precision, a, B, 0, symbol_len - 1, st, nullptr);
}

int32_t ofs_minn_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                        int32_t symbol_len, int32_t precision, void* M, void* P, void* R,
                        void* stream) {
    if (!fmt_ok(in_fmt) || !prec_ok(precision) || OFS_MISSING(x, B * T) || B < 0 || n_br < 1 || T < 0 || symbol_len < 1)
        return OFS_EINVAL;
    const int64_t n_out = T - symbol_len + 1;
    if (B == 0 || n_out <= 0) return OFS_OK;
    {
        const WinFastArgs f{x, B, T, symbol_len, M, P, R};
        const int frc = ofs_win_fast_try(3, in_fmt, precision, n_br, f, (hipStream_t)stream);
        if (frc != 0) return frc > 0 ? OFS_OK : frc;
    }
    WinArgs a{};
    a.x = x; a.T = T; a.n_out = n_out; a.nb = n_br; a.Q = symbol_len / 4; a.D = symbol_len / 4;
    a.N = symbol_len; a.P = P; a.R = R; a.M = M;
    return dispatch_win<M_MINN>(in_fmt, precision, a, B, 0, symbol_len - 1, (hipStream_t)stream, nullptr);
}

int32_t ofs_minn_rtl(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                     int32_t Q, int32_t smooth_shift, int32_t smooth_mode,
                     int64_t threshold_value, int32_t threshold_frac_bits,
                     double* corr_total, double* corr_positive, double* smooth_metric,
                     double* energy_total, double* corr_scaled, double* energy_scaled,
                     uint8_t* metric_valid, uint8_t* above_threshold,
                     int32_t detect, int32_t hysteresis, int32_t timing_offset,
                     int32_t max_events, int32_t* n_events, int64_t* events,
                     int64_t* open_gate_start, void* stream) {
    if (!(fmt_ok(in_fmt) || in_fmt == OFS_CP12) || OFS_MISSING(x, B * T) || B < 0 || n_br < 1 || T < 0 || Q < 1)
        return OFS_EINVAL;
    if (OFS_MISSING(corr_total, B * T) || OFS_MISSING(energy_total, B * T) || smooth_shift < 0 || smooth_shift > 62 ||
        threshold_frac_bits < 0 || threshold_frac_bits > 62 || (smooth_mode != 0 && smooth_mode != 1))
        return OFS_EINVAL;
    if (detect && (OFS_MISSING(n_events, B) || max_events < 0 || (max_events > 0 && OFS_MISSING(events, B))))
        return OFS_EINVAL;
    if (B == 0 || T == 0) return OFS_OK;
    if (3 * (int64_t)Q - 1 > 0x3fffffff) return OFS_ETOOLONG;
    hipStream_t st = (hipStream_t)stream;
    {   // int16 I/Q: exact wave-per-stream kernel, metric + smoothing + gate in one pass
        RtlExactCall c{};
        c.x = x; c.B = B; c.T = T; c.Q = Q; c.shift = smooth_shift; c.smooth_mode = smooth_mode;
        c.frac_bits = threshold_frac_bits; c.thr_value = (double)threshold_value;
        c.corr_total = corr_total; c.corr_positive = corr_positive; c.smooth = smooth_metric;
        c.energy_total = energy_total; c.corr_scaled = corr_scaled; c.energy_scaled = energy_scaled;
        c.mvalid = metric_valid; c.above = above_threshold; c.detect = detect; c.hyst = hysteresis;
        c.toff = timing_offset; c.max_ev = max_events; c.n_ev = n_events; c.ev = events;
        c.open_start = open_gate_start;
        const int frc = ofs_rtl_exact_try(in_fmt, n_br, c, st);
        if (frc == 1) return OFS_OK;
        if (frc < 0) return frc;
    }
    if (in_fmt == OFS_CP12) return OFS_EINVAL;                        // packed words: exact kernel only
    WinArgs a{};
    a.x = x; a.T = T; a.n_out = T; a.nb = n_br; a.Q = Q; a.D = Q; a.W = Q;
    a.corr_total = corr_total; a.corr_positive = corr_positive; a.energy_total = energy_total;
    a.energy_scaled = energy_scaled; a.mvalid = metric_valid; a.thr_value = (double)threshold_value;
    int rc = dispatch_win<M_RTL>(in_fmt, OFS_FP64, a, B, -(3 * Q - 1), 0, st, nullptr);
    if (rc) return rc;
    if (smooth_metric || corr_scaled || above_threshold || detect) {
        RtlArgs r{};
        r.corr_total = corr_total; r.energy_total = energy_total; r.smooth = smooth_metric;
        r.corr_scaled = corr_scaled; r.above = above_threshold; r.T = T; r.Q = Q;
        r.shift = smooth_shift; r.smooth_mode = smooth_mode; r.frac_bits = threshold_frac_bits;
        r.thr_value = (double)threshold_value; r.detect = detect; r.hyst = hysteresis;
        r.toff = timing_offset; r.max_ev = max_events; r.n_ev = n_events; r.ev = events;
        r.open_start = open_gate_start;
        hipLaunchKernelGGL(rtl_iir_kernel, dim3((unsigned)((B + 63) / 64)), dim3(256), 0, st, r, B);
        if (hipGetLastError() != hipSuccess) return OFS_EHIP;
    }
    return OFS_OK;
}

int32_t ofs_rtl_plan(int32_t in_fmt, int32_t n_br, int64_t T, int32_t Q) {
    const int xp = ofs_rtl_exact_plan(in_fmt, n_br, T, Q);
    return xp ? 2000 + xp : 0;
}

int32_t ofs_minn_rtl_gate(const double* corr_positive, const uint8_t* above_threshold,
                          const uint8_t* metric_valid, int64_t B, int64_t T,
                          int32_t hysteresis, int32_t timing_offset, int32_t max_events,
                          int32_t* n_events, int64_t* events, int64_t* open_gate_start,
                          void* stream) {
    if (!corr_positive || !above_threshold || !metric_valid || !n_events || B < 0 || T < 0 ||
        max_events < 0 || (max_events > 0 && !events))
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipLaunchKernelGGL(rtl_gate_kernel, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream,
                       corr_positive, above_threshold, metric_valid, T, hysteresis, timing_offset,
                       max_events, n_events, events, open_gate_start);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_sc_minn_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                           int32_t symbol_len, int32_t precision, void* M_sc, void* P_sc, void* R_sc,
                           void* M_minn, void* P_minn, void* R_minn, void* stream) {
    if (!fmt_ok(in_fmt) || !prec_ok(precision) || OFS_MISSING(x, B * T) || B < 0 || n_br < 1 || T < 0 || symbol_len < 2 ||
        (symbol_len & 1))
        return OFS_EINVAL;
    if (B == 0 || T - symbol_len + 1 <= 0) return OFS_OK;
    hipStream_t st = (hipStream_t)stream;
    const int frc = ofs_sc_minn_fast_try(in_fmt, precision, n_br, x, B, T, symbol_len, M_sc, P_sc, R_sc,
                                         M_minn, P_minn, R_minn, st);
    if (frc != 0) return frc > 0 ? OFS_OK : frc;
    const int rc = ofs_sc_metric(in_fmt, x, B, n_br, T, symbol_len, 1, precision, M_sc, P_sc, R_sc, stream);
    if (rc) return rc;
    return ofs_minn_metric(in_fmt, x, B, n_br, T, symbol_len, precision, M_minn, P_minn, R_minn, stream);
}

int32_t ofs_win_plan(int32_t kind, int32_t in_fmt, int32_t precision, int32_t n_br, int64_t T,
                     int32_t symbol_len) {
    if (kind == 4) return ofs_sc_minn_fast_plan(in_fmt, precision, n_br, T, symbol_len);
    return ofs_win_fast_plan(kind, in_fmt, precision, n_br, T, symbol_len);
}

int32_t ofs_cp_cfo(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                   const int64_t* starts, int32_t n_fft, int32_t cp_len, double fs_hz,
                   double* P_out, double* cfo_out, void* stream) {
    if (!fmt_ok(in_fmt) || OFS_MISSING(x, B * T) || OFS_MISSING(starts, B) || OFS_MISSING(cfo_out, B) || B < 0 ||
        n_br < 1 || T < 0 || n_fft < 1 || cp_len < 0)
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipStream_t st = (hipStream_t)stream;
    switch (in_fmt) {
        case OFS_C64:
            hipLaunchKernelGGL(cp_cfo_kernel<OFS_C64>, dim3((unsigned)B), dim3(WG), 0, st, x, T, n_br, starts, n_fft, cp_len, fs_hz, P_out, cfo_out);
            break;
        case OFS_C128:
            hipLaunchKernelGGL(cp_cfo_kernel<OFS_C128>, dim3((unsigned)B), dim3(WG), 0, st, x, T, n_br, starts, n_fft, cp_len, fs_hz, P_out, cfo_out);
            break;
        default:
            hipLaunchKernelGGL(cp_cfo_kernel<OFS_CI16>, dim3((unsigned)B), dim3(WG), 0, st, x, T, n_br, starts, n_fft, cp_len, fs_hz, P_out, cfo_out);
    }
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

}  // extern "C"

namespace ofs {
int64_t variant(Variant v) {
    return g_variants.v[v];
}
}  // namespace ofs
