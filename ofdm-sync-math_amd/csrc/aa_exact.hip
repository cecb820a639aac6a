// aa_exact.hip — integer-exact wave-per-stream kernels for int16 I/Q input (OFS_CI16: 12-bit ADC
// words, the RTL's sample format, ref/minn_preamble_detector.sv:61-67):
//
//   aa_exact_kernel  [A][A] S&C detector: P, R, M, valid + gate / peak / CFO events
//                    (sync_aa.py:421-571), fp64 outputs;
//   rtl_exact_kernel RTL Minn metric (minn_rtl.py:583-733) fused with the IIR smoothing,
//                    threshold and gate FSM (minn_rtl.py:706-722, :750-825).
//
// Every product and window sum of integer samples is an integer below 2^53 (checked on the
// host: T·n_branch <= 2^21), so fp64 PREFIX DIFFERENCES ARE EXACT: any summation order gives the
// bits of the reference's sequential running sums.  No cancellation-free split is needed
// (contrast aa_fast.hip), which makes this the cheap path: one wave per stream, rows of
// RL = 64·E samples (lane l owns samples RL·k + E·l + e), the lagged sample and the lagged
// prefix values sit in the same lane and element a whole number of rows back.
//
// The RTL smoothing s += (c - s) / 2^k is the reference's float64 recursion and is sequential in
// time; it runs inside the same wave, row by row, on wave-uniform values (v_readlane of the
// row's corr_positive), so the metric never makes a round trip through HBM before smoothing.
#include "ofs_common.h"
#include "aa_gate.h"
#include "ofdmsync.h"

using namespace ofs;

namespace {

constexpr int XW = 256;                 // 4 waves = 4 streams per workgroup
#ifndef OFS_XA_WG
#define OFS_XA_WG 256
#endif
#ifndef OFS_XWPE1                   // min waves per SIMD of the integer L = RL kernels (tuning builds)
#define OFS_XWPE1 1
#endif
#ifndef OFS_XPD1                    // their rows in flight ahead of use (tuning builds)
#define OFS_XPD1 4
#endif
constexpr int XA = OFS_XA_WG;           // aa_exact_kernel workgroup (tuning builds: 64)
// workgroup of one instantiation: the integer L = RL one-antenna kernel (cfg2a) runs one stream per
// workgroup - paired (round 6, profiles/r06y_exact_wg_ab.txt): cfg2a 0.0283 -> 0.0273 ms, packed AXIS
// words 0.0322 -> 0.0313; complex128 keeps 4 (cfg3_fp64 0.5895 vs 0.6106 ms at 1, the 2 x 5315 fp64
// shape 1.1348 vs 1.1473)
#ifndef OFS_XA_WG_I1
#define OFS_XA_WG_I1 64
#endif
constexpr int xa_wg(int fmt, int mr, int na) { return (fmt != OFS_C128 && mr == 1 && na == 1) ? OFS_XA_WG_I1 : XA; }

// E consecutive int16 I/Q words (packed (I, Q) in one int32) of one lane, zero past T
template <int E>
__device__ __forceinline__ void load_words(const int32_t* xs, int64_t n0, int64_t T, int32_t (&w)[E]) {
    if (n0 + E <= T && (reinterpret_cast<uintptr_t>(xs + n0) & (4 * E - 1)) == 0) {
        if constexpr (E == 1) {
            w[0] = xs[n0];
        } else if constexpr (E == 2) {
            const int2 v = *reinterpret_cast<const int2*>(xs + n0);
            w[0] = v.x; w[1] = v.y;
        } else {
#pragma unroll
            for (int j = 0; j < E; j += 4) {
                const int4 v = *reinterpret_cast<const int4*>(xs + n0 + j);
                w[j] = v.x; w[j + 1] = v.y; w[j + 2] = v.z; w[j + 3] = v.w;
            }
        }
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) w[e] = (n0 + e < T) ? xs[n0 + e] : 0;
    }
}
// OFS_CP12: E consecutive time indices n0.. of the NA channels of one stream (base x8), decoded
// to the int16 I/Q words above.  Fast path: the lane's 3·NA·E bytes with dword loads from the
// dword below, realigned with v_alignbyte (groups then sit at compile-time byte offsets); used
// when the row is whole and the rounded-up dword window stays inside the buffer.  Otherwise per
// byte with zero fill past T.
__device__ __forceinline__ int32_t cp12_word(uint32_t g) {
    const int32_t i = ((int32_t)(g << 20)) >> 20;              // bits 0-11, sign-extended
    const int32_t q = ((int32_t)(g << 8)) >> 20;               // bits 12-23
    return (i & 0xffff) | (int32_t)((uint32_t)q << 16);
}
template <int E, int NA>
__device__ __forceinline__ void cp12_load(const uint8_t* x8, int64_t sbyte, int64_t n0, int64_t T, int64_t total,
                                          int32_t (&w)[NA][E]) {
    constexpr int NB = 3 * NA * E;                              // bytes wanted
    constexpr int ND = (NB + 3 + 3) / 4;                        // dwords covering them at any shift
    const int64_t p = sbyte + 3 * NA * n0;                      // absolute byte offset in the buffer
    const int64_t a = p & ~(int64_t)3;
    if (n0 + E <= T && a + 4 * ND <= total) {
        const uint32_t* d = reinterpret_cast<const uint32_t*>(x8 - sbyte + a);
        uint32_t v[ND];
#pragma unroll
        for (int j = 0; j < ND; ++j) v[j] = d[j];
        const uint32_t sh = (uint32_t)(p & 3);
        uint32_t al[ND - 1];                                    // bytes p, p+1, ... in order
#pragma unroll
        for (int j = 0; j + 1 < ND; ++j) al[j] = __builtin_amdgcn_alignbyte(v[j + 1], v[j], sh);
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
            for (int t = 0; t < NA; ++t) {
                const int bo = 3 * (e * NA + t);                // compile-time after unrolling
                const uint64_t win = ((uint64_t)al[bo / 4 + 1 < ND - 1 ? bo / 4 + 1 : ND - 2] << 32) | al[bo / 4];
                w[t][e] = cp12_word((uint32_t)(win >> (8 * (bo & 3))) & 0xffffffu);
            }
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
            for (int t = 0; t < NA; ++t) {
                if (n0 + e < T) {
                    const uint8_t* q = x8 + 3 * (NA * (n0 + e) + t);
                    w[t][e] = cp12_word((uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16));
                } else {
                    w[t][e] = 0;
                }
            }
    }
}

__device__ __forceinline__ double w_re(int32_t w) { return (double)(int16_t)(w & 0xffff); }
__device__ __forceinline__ double w_im(int32_t w) { return (double)(w >> 16); }

// sample access of the wave-per-stream sync_aa kernel: int16 I/Q words (exact integer sums) or
// complex128 (fp64 prefix differences over the stream, the general engine's arithmetic)
template <int FMT> struct XSamp;
template <> struct XSamp<OFS_CI16> {
    using W = int32_t;
    static __device__ __forceinline__ W zero() { return 0; }
    static __device__ __forceinline__ double re(W w) { return w_re(w); }
    static __device__ __forceinline__ double im(W w) { return w_im(w); }
    template <int E>
    static __device__ __forceinline__ void load(const W* xs, int64_t n0, int64_t T, W (&w)[E]) {
        load_words<E>(xs, n0, T, w);
    }
};
template <> struct XSamp<OFS_C128> {
    using W = double2;
    static __device__ __forceinline__ W zero() { return make_double2(0.0, 0.0); }
    static __device__ __forceinline__ double re(W w) { return w.x; }
    static __device__ __forceinline__ double im(W w) { return w.y; }
    template <int E>
    static __device__ __forceinline__ void load(const W* xs, int64_t n0, int64_t T, W (&w)[E]) {
#pragma unroll
        for (int e = 0; e < E; ++e) w[e] = (n0 + e < T) ? xs[n0 + e] : zero();
    }
};

// in-lane inclusive prefix of v, then the lane's exclusive wave prefix and the row total
template <int E>
struct RowPrefix {
    double f[E], excl, tot;
    __device__ __forceinline__ void run(const double (&v)[E]) {
        f[0] = v[0];
#pragma unroll
        for (int e = 1; e < E; ++e) f[e] = f[e - 1] + v[e];
        const double incl = scan_add(f[E - 1]);
        excl = shr1z(incl);
        tot = readlane(incl, 63);
    }
};

// The same row prefix on int32 values (integer-valued products of 12-bit words: a row of 64·E
// samples of one or two branches stays below 2^31), exactly the doubles' values
template <int E>
struct RowPrefixI {
    int f[E], excl, tot;
    __device__ __forceinline__ void run(const int (&v)[E]) {
        f[0] = v[0];
#pragma unroll
        for (int e = 1; e < E; ++e) f[e] = f[e - 1] + v[e];
        const int incl = scan_add_i32(f[E - 1]);
        excl = dppz_i<0x138>(incl);                   // wave_shr:1, lane 0 <- 0
        tot = __builtin_amdgcn_readlane(incl, 63);
    }
};

// ------------------------------------------------------------------------------------------
// sync_aa, integer input (FMT = OFS_CI16, exact) or complex128 (OFS_C128, any T: stream-wide fp64
// prefix differences, the reference's running-sum error regime; see ofs_aa_exact_plan).  P[n] = A(n) - A(n-L), R[n] = Ae(n) - Ae(n-L) with A the prefix of
// x[j]·conj(x[j-L]) (0 while the delay line fills) and Ae that of |x[j]|², summed over antennas;
// valid = n >= L; M = min(|P|²/R², 1) if valid and R > 1e-6·L else 0 (sync_aa.py:458-493).
// ------------------------------------------------------------------------------------------
template <int FMT, int E, int MR, int NA>
__global__ __launch_bounds__(xa_wg(FMT, MR, NA), (FMT == OFS_C128 && MR == 4 && NA == 1) ? 2 : (FMT != OFS_C128 && MR == 1 && NA == 1 ? OFS_XWPE1 : 1)) void aa_exact_kernel(AaFastArgs a) {
    using X = XSamp<FMT == OFS_CP12 ? OFS_CI16 : FMT>;          // CP12 decodes to int16 I/Q words
    using W = typename X::W;
    constexpr int RL = 64 * E;
    constexpr int L = MR * RL;
    constexpr int PD = (FMT != OFS_C128 && MR == 1 && NA == 1) ? OFS_XPD1 : (E <= 2 ? 4 : 2);   // rows in flight ahead of use
    constexpr int PER = MR > PD ? MR : PD;                   // unroll period (MR, PD powers of 2)
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)xcd_block_w() * (xa_wg(FMT, MR, NA) / 64) + (threadIdx.x >> 6);
    if (b >= a.B) return;
    const int64_t T = a.T;
    const int nrows = (int)((T + RL - 1) / RL);
    const W* xs = reinterpret_cast<const W*>(a.x) + b * NA * T;
    const int64_t sbyte = b * NA * T * 3;                        // CP12: stream start in bytes
    const uint8_t* x8 = reinterpret_cast<const uint8_t*>(a.x) + sbyte;
    const int64_t total = a.B * NA * T * 3;
    auto load_all = [&](int64_t n0, W (&dst)[NA][E]) {
        if constexpr (FMT == OFS_CP12) {
            cp12_load<E, NA>(x8, sbyte, n0, T, total, dst);
        } else {
#pragma unroll
            for (int t = 0; t < NA; ++t) X::template load<E>(xs + t * T, n0, T, dst[t]);
        }
    };

    W lag[NA][MR][E];                                        // raw samples of rows k-MR..k-1
    double Ar[MR][E], Ai[MR][E], Ae[MR][E];                  // prefix values of rows k-MR..k-1
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int e = 0; e < E; ++e) {
            Ar[m][e] = 0.0; Ai[m][e] = 0.0; Ae[m][e] = 0.0;
#pragma unroll
            for (int t = 0; t < NA; ++t) lag[t][m][e] = X::zero();
        }
    double CR = 0.0, CI = 0.0, CE = 0.0;                     // prefix at the start of row k

    W nx[PD][NA][E];
#pragma unroll
    for (int p = 0; p < PD; ++p) load_all((int64_t)RL * p + E * lane, nx[p]);

    AaRowGate<E, double, false, true, FMT != OFS_C128> gate;
    if (a.detect)
        gate.init(a.hyst, L, a.thr, a.fs, a.max_ev, a.ev_i + b * (int64_t)a.max_ev * 4,
                  a.ev_r + b * (int64_t)a.max_ev * 4);
    double2* Pout = reinterpret_cast<double2*>(a.P) + b * T;
    double* Rout = reinterpret_cast<double*>(a.R) + b * T;
    double* Mout = reinterpret_cast<double*>(a.M) + b * T;
    uint8_t* Vout = a.valid ? a.valid + b * T : nullptr;
    const double floor_ = 1e-6 * (double)L;

    for (int k0 = 0; k0 < nrows; k0 += PER) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = k0 + u;
            if (k < nrows) {
                const int nb = RL * k + E * lane;
                W cur[NA][E];
#pragma unroll
                for (int t = 0; t < NA; ++t)
#pragma unroll
                    for (int e = 0; e < E; ++e) cur[t][e] = nx[u % PD][t][e];
                if (k + PD < nrows) load_all((int64_t)RL * (k + PD) + E * lane, nx[u % PD]);
                const int sl = u % MR;                       // ring slot of row k-MR (and k)
                double pr[E], pi[E], en[E];
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    pr[e] = 0.0; pi[e] = 0.0; en[e] = 0.0;
#pragma unroll
                    for (int t = 0; t < NA; ++t) {
                        const double xr = X::re(cur[t][e]), xi = X::im(cur[t][e]);
                        const double dr = X::re(lag[t][sl][e]), di = X::im(lag[t][sl][e]);
                        pr[e] += xr * dr + xi * di;                  // x[n]·conj(x[n-L]), exact
                        pi[e] += xi * dr - xr * di;
                        en[e] += xr * xr + xi * xi;
                        lag[t][sl][e] = cur[t][e];
                    }
                }
                RowPrefix<E> qr, qi, qe;
                qr.run(pr); qi.run(pi); qe.run(en);
                double oP[E][2], oR[E], oM[E], opm[E];
                const bool valid = k >= MR;                          // n >= L for the whole row
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const double A_r = (CR + qr.excl) + qr.f[e];
                    const double A_i = (CI + qi.excl) + qi.f[e];
                    const double A_e = (CE + qe.excl) + qe.f[e];
                    const double Pr = A_r - Ar[sl][e], Pi = A_i - Ai[sl][e], Rr = A_e - Ae[sl][e];
                    Ar[sl][e] = A_r; Ai[sl][e] = A_i; Ae[sl][e] = A_e;
                    const double pm = Pr * Pr + Pi * Pi;
                    double m = 0.0;
                    if (valid && Rr > floor_) { m = pm / (Rr * Rr); m = m < 1.0 ? m : 1.0; }
                    oP[e][0] = Pr; oP[e][1] = Pi; oR[e] = Rr; oM[e] = m; opm[e] = pm;
                }
                CR += qr.tot; CI += qi.tot; CE += qe.tot;
                // stores: a lane's E samples are contiguous
                const bool whole = nb + E <= T && ((T & 1) == 0);
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (a.P && nb + e < T) Pout[nb + e] = make_double2(oP[e][0], oP[e][1]);
                if (whole && E >= 2) {
#pragma unroll
                    for (int e = 0; e < E; e += 2) {
                        if (a.R) *reinterpret_cast<double2*>(Rout + nb + e) = make_double2(oR[e], oR[e + 1]);
                        if (a.M) *reinterpret_cast<double2*>(Mout + nb + e) = make_double2(oM[e], oM[e + 1]);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < E; ++e)
                        if (nb + e < T) {
                            if (a.R) Rout[nb + e] = oR[e];
                            if (a.M) Mout[nb + e] = oM[e];
                        }
                }
                if (Vout) {
#pragma unroll
                    for (int e = 0; e < E; ++e)
                        if (nb + e < T) Vout[nb + e] = (uint8_t)valid;
                }
                if (a.detect && valid) {
                    double ppr[E], ppi[E];
#pragma unroll
                    for (int e = 0; e < E; ++e) { ppr[e] = oP[e][0]; ppi[e] = oP[e][1]; }
                    gate.row(lane, k, nb, (int)T, oM, opm, ppr, ppi);
                }
            }
        }
    }
    if (a.detect) gate.finish(lane, (int)T, a.n_ev + b);
}

// ------------------------------------------------------------------------------------------
// minn_rtl, integer input.  With Ac / Ae the prefixes of the lag-Q real product
// Re(x[j]·conj(x[j-Q])) (0 while the delay line fills) and of |x[j]|², summed over branches,
// and Q-windows C(i) = Ac(i) - Ac(i-Q), En(i) = Ae(i) - Ae(i-Q) (the _antenna_path registers
// hold 0 until their first valid sample):
//   corr_total   = [i >= Q-1] C(i) + [i >= 2Q-1] C(i-Q)
//   energy_total = [i >= Q-1] En(i) + [i >= 2Q-1] En(i-Q) + [i >= 3Q-1] En(i-2Q)
//   metric_valid = i >= 3Q-1                                  (minn_rtl.py:609-643, :691-702)
// The lagged prefixes (Q, 2Q, 3Q back) live in a per-wave LDS ring of rows.
// ------------------------------------------------------------------------------------------
struct RtlExactArgs {
    const void* x; int64_t B, T; int32_t nb, Q;
    int32_t shift, smooth_mode, frac_bits; double thr_value;
    double* corr_total; double* corr_positive; double* smooth; double* energy_total;
    double* corr_scaled; double* energy_scaled; uint8_t* mvalid; uint8_t* above;
    int32_t detect, hyst, toff, max_ev; int32_t* n_ev; int64_t* ev; int64_t* open_start;
};

// ---- segment-parallel smoothing -----------------------------------------------------------
// The stream is cut into segments of SEG = 64·SC samples; lane j owns the chunk of SC samples
// [s0 + SC·j, s0 + SC·(j+1)).  The float IIR s <- s + (c - s)·2^-k (minn_rtl.py:706-715) is
// evaluated EXACTLY - the reference's sequential operation sequence, contraction off - by
// every lane over its own chunk, from an entering state that is made self-consistent:
//   1. guess: each lane maps its chunk from s = 0 and records the affine map s_out = A·s_in + Z;
//      a wave scan of the maps applied to the exact carried state gives every chunk's
//      entering state to a few ulps;
//   2. round: every lane runs the exact recursion over its chunk from its entering state; the
//      chain is consistent when each lane's entering state equals lane j-1's leaving state
//      bit for bit (lane 0 enters with the exact carried state).  Otherwise every lane takes
//      lane j-1's leaving state as its new entering state and the round repeats.
// The recursion is deterministic, so a consistent chain IS the reference's trajectory (by
// induction from lane 0).  After round r lanes 0..r are exact, so it ends within 64 rounds
// (the sequential cost); in practice the guessed trajectories coincide with the exact one
// inside a chunk or two and a segment takes a few rounds.  The integer floor-shift RTL mode
// (not contractive to the bit) runs in a walker lane per stream instead (rtl_walk).
#ifndef OFS_RTL_SC
#define OFS_RTL_SC 4
#endif
constexpr int SC = OFS_RTL_SC;
static_assert(SC % 2 == 0, "chunk stores go out as 16-byte pairs");
constexpr int SEG = 64 * SC;
constexpr int SEG_PAD = SEG + SEG / SC;                // chunk stride SC + 1 doubles (banks)
__device__ __forceinline__ int seg_at(int i) { return i + i / SC; }

// per-wave LDS: prefix rows k-3MW..k of Ae and Ac, the raw words of rows k-MW..k-1 of every
// branch (lane-private columns), the segment's corr_positive and energy_scaled
__host__ __device__ constexpr int rtl_ring_rows(int MW) { return 3 * MW + 1; }
__host__ __device__ constexpr size_t rtl_wave_lds(int E, int MW, int nb) {
    return (size_t)2 * rtl_ring_rows(MW) * E * 64 * sizeof(double) + (size_t)2 * SEG_PAD * sizeof(double) +
           (size_t)nb * MW * E * 64 * sizeof(int32_t);
}

__device__ __forceinline__ bool same_bits(double a, double b) {
    return __double_as_longlong(a) == __double_as_longlong(b);
}

// One walker lane's pass over a segment (phase B below): the reference's IIR (minn_rtl.py:706-715)
// exactly as written, branch-free per sample, SM = 0 float s += (c - s)/2^k, 1 shift 0 (s = c),
// 2 RTL floor shift; the threshold decision (:717-722) goes into the stored value's sign bit.
template <int SM>
__device__ __forceinline__ void rtl_walk(const double* __restrict__ wcp, double* __restrict__ wes, int n, int v0,
                                         double inv, double scale, int shift, double& sv, long long& siv) {
    constexpr long long SIGN = (long long)(1ull << 63);
    auto step = [&](double c, double es) -> double {
        if constexpr (SM == 0) sv = sv + (c - sv) * inv;
        else if constexpr (SM == 1) sv = c;
        else {
            const long long ci = (long long)c;
            siv = shift == 0 ? ci : siv + ((ci - siv) >> shift);
            sv = (double)siv;
        }
        return __longlong_as_double(__double_as_longlong(sv) | (sv * scale >= es ? SIGN : 0ll));
    };
    int li = 0;
    for (; li < v0; ++li) wes[seg_at(li)] = sv;                  // before metric_valid: state held
    for (; li + 8 <= n; li += 8) {
        double cb[8], eb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { cb[u] = wcp[seg_at(li + u)]; eb[u] = wes[seg_at(li + u)]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) wes[seg_at(li + u)] = step(cb[u], eb[u]);
    }
    for (; li < n; ++li) wes[seg_at(li)] = step(wcp[seg_at(li)], wes[seg_at(li)]);
}

// workgroup barrier ordering LDS only: a __syncthreads() fence would also wait for every global
// store in flight (vmcnt(0)), a store round trip per segment
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int E, int MW, int CPNA, int NBM>
__global__ __launch_bounds__(XW) void rtl_exact_kernel(RtlExactArgs a) {
#pragma clang fp contract(off)
    constexpr int RL = 64 * E;
    constexpr int Q = MW * RL;
    constexpr int NR = rtl_ring_rows(MW);
    static_assert(SEG % RL == 0, "segment = whole metric rows");
    extern __shared__ __attribute__((aligned(16))) double rsm[];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    const int64_t b = (int64_t)blockIdx.x * wpb + w;
    const int64_t T = a.T;
    const int nb_ = a.nb;
    const bool seq = a.smooth || a.corr_scaled || a.above || a.detect;
    const size_t wave_dbl = rtl_wave_lds(E, MW, nb_) / sizeof(double);
    const int smode = a.smooth_mode == 1 ? 2 : (a.shift == 0 ? 1 : 0);
#ifndef OFS_RTL_WALK_ALL                    // tuning builds: every smoothing mode in the walker
#define OFS_RTL_WALK_ALL 0
#endif
    const bool walk = seq && (smode == 2 || OFS_RTL_WALK_ALL);   // RTL floor IIR: walker lane (barriers)
    if (b >= a.B) {                 // no stream: still meet the workgroup's two barriers per segment
        if (walk)
            for (int64_t g = 0; g < (T + SEG - 1) / SEG; ++g) { lds_barrier(); lds_barrier(); }
        return;
    }
    double* hae_ = rsm + wave_dbl * w;
    double* hac_ = hae_ + NR * E * 64;
    double* hcp = hac_ + NR * E * 64;                                // segment corr_positive
    double* hes = hcp + SEG_PAD;                                     // segment energy_scaled
    int32_t* hx_ = reinterpret_cast<int32_t*>(hes + SEG_PAD);
    auto hae = [&](int r, int e) -> double& { return hae_[(r * E + e) * 64 + lane]; };
    auto hac = [&](int r, int e) -> double& { return hac_[(r * E + e) * 64 + lane]; };
    auto hx = [&](int t, int m, int e) -> int32_t& { return hx_[((t * MW + m) * E + e) * 64 + lane]; };
    const int nrows = (int)((T + RL - 1) / RL);
    const int32_t* xs = reinterpret_cast<const int32_t*>(a.x) + b * nb_ * T;
    const int64_t sbyte = b * nb_ * T * 3;                         // CP12 (CPNA branches)
    const uint8_t* x8 = reinterpret_cast<const uint8_t*>(a.x) + sbyte;
    const int64_t total = a.B * nb_ * T * 3;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int e = 0; e < E; ++e) { hae(r, e) = 0.0; hac(r, e) = 0.0; }
    for (int t = 0; t < nb_; ++t)
#pragma unroll
        for (int m = 0; m < MW; ++m)
#pragma unroll
            for (int e = 0; e < E; ++e) hx(t, m, e) = 0;

    const int64_t row_off = b * T;
    const bool vec_st = (T % SC) == 0 && (reinterpret_cast<uintptr_t>(a.above) & 3) == 0 &&
                        ((reinterpret_cast<uintptr_t>(a.smooth) | reinterpret_cast<uintptr_t>(a.corr_scaled)) & 7) == 0;
    const int vstart = 3 * Q - 1;
    const double inv = ldexp(1.0, -(a.shift > 0 ? a.shift : 0));   // exact 1 / 2^shift
    const double keep = 1.0 - inv;
    const double scale = (double)(1ll << a.frac_bits);
    double CC = 0.0, CE = 0.0;
    bool wide = false;                                             // a word beyond 12 bits seen (sticky)
    double sm = 0.0;                                               // IIR state carried between segments
    long long si = 0;
#if OFS_RTL_ROUNDS_DEBUG
    long long dbg_rounds = 0;
#endif
    AaRowGate<SC, double, true, true, false> gate;                 // detect_minn_rtl, closed form
    if (a.detect)
        gate.init(a.hyst, Q, 0.0, 0.0, a.max_ev, a.ev ? a.ev + b * (int64_t)a.max_ev * 4 : nullptr,
                  nullptr, a.toff);

    // Rows arrive one segment ahead of use: segment g+1's RPS rows are loaded when segment g takes its
    // own.  gfx9 counts loads and stores on one counter (vmcnt), in issue order, so the first use of
    // a loaded register also waits for every store the wave issued before that load.  A segment
    // therefore takes all its rows at once, before it issues any store, and its phase-C stores go out after the next segment has taken its rows: the one wait per segment
    // finds only long-issued operations in flight.  (A queue shifted by one row per step waited on
    // every row for the previous row's stores.)
    constexpr int RPS = SEG / RL;
    // NBM: branches held per row (1, or 4 = the most supported; CPNA > 0: CPNA)
    int32_t nx[RPS][NBM][E];
    // one row of every branch (CPNA > 0: packed 12-bit words, CPNA branches)
    auto load_row = [&](int64_t n0, int32_t (&dst)[NBM][E]) {
        if constexpr (CPNA > 0) {
            int32_t w[CPNA][E];
            cp12_load<E, CPNA>(x8, sbyte, n0, T, total, w);
#pragma unroll
            for (int t = 0; t < NBM; ++t)
#pragma unroll
                for (int e = 0; e < E; ++e) dst[t][e] = t < CPNA ? w[t < CPNA ? t : 0][e] : 0;
        } else {
#pragma unroll
            for (int t = 0; t < NBM; ++t) {
                if (t < nb_) load_words<E>(xs + t * T, n0, T, dst[t]);
                else
#pragma unroll
                    for (int e = 0; e < E; ++e) dst[t][e] = 0;
            }
        }
    };
    auto load_seg = [&](int g) {
#pragma unroll
        for (int j = 0; j < RPS; ++j)
            if (g * RPS + j < nrows) load_row((int64_t)RL * (g * RPS + j) + E * lane, nx[j]);
    };
    load_seg(0);
    // phase-C stores of a lane's chunk (issued one segment late, see above)
    auto store_chunk = [&](int64_t c0, const double (&own)[SC], const bool (&abv)[SC]) {
        if (vec_st && c0 + SC <= T) {
            // whole chunk (T % SC == 0, flag buffer dword-aligned): 16-byte stores, one packed flag word
            const int64_t gi = row_off + c0;
#pragma unroll
            for (int e = 0; e < SC; e += 2) {
                if (a.smooth) *reinterpret_cast<double2*>(a.smooth + gi + e) = make_double2(own[e], own[e + 1]);
                if (a.corr_scaled)
                    *reinterpret_cast<double2*>(a.corr_scaled + gi + e) = make_double2(own[e] * scale, own[e + 1] * scale);
            }
            if (a.above) {
                if constexpr (SC == 4) {
                    *reinterpret_cast<uint32_t*>(a.above + gi) =
                        (uint32_t)abv[0] | ((uint32_t)abv[1] << 8) | ((uint32_t)abv[2] << 16) | ((uint32_t)abv[3] << 24);
                } else {
#pragma unroll
                    for (int e = 0; e < SC; ++e) a.above[gi + e] = (uint8_t)abv[e];
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < SC; ++e) {
                const int64_t p = c0 + e;
                if (p < T) {
                    const int64_t gi = row_off + p;
                    if (a.smooth) a.smooth[gi] = own[e];
                    if (a.corr_scaled) a.corr_scaled[gi] = own[e] * scale;
                    if (a.above) a.above[gi] = (uint8_t)abv[e];
                }
            }
        }
    };
    bool pend = false;                                             // a chunk's stores deferred
    int64_t pend_c0 = 0;
    double pend_own[SC];
    bool pend_abv[SC];

    const int nseg = (int)((T + SEG - 1) / SEG);
    for (int g = 0; g < nseg; ++g) {
        const int64_t s0 = (int64_t)SEG * g;
        const int k0 = g * RPS, k1 = min(nrows, (g + 1) * RPS);
        int32_t rows[RPS][NBM][E];                                 // the segment's rows, taken at once
#pragma unroll
        for (int j = 0; j < RPS; ++j)
#pragma unroll
            for (int t = 0; t < NBM; ++t)
#pragma unroll
                for (int e = 0; e < E; ++e) rows[j][t][e] = nx[j][t][e];
        if (g + 1 < nseg) load_seg(g + 1);
        if (pend) { store_chunk(pend_c0, pend_own, pend_abv); pend = false; }
        // ---------------- phase A: metric rows of the segment (stores of the metric arrays) ----
#pragma unroll
        for (int j = 0; j < RPS; ++j) {
            const int k = k0 + j;
            if (k >= k1) break;
            const int nb = RL * k + E * lane;
            const int xsl = k % MW;
            const int32_t (&cur)[NBM][E] = rows[j];
            // Products and energies of 12-bit words are integers below 2^23 per sample and branch: for
            // <= 2 branches a row's prefix stays below 2^31 (2 x 2^23 x 64·E), so while every word seen
            // so far is 12-bit (sticky, wave-uniform check; int16 input may carry wider words) the row
            // scans run in int32 (one DPP add per step instead of three instructions per fp64 step):
            // the same integer values exactly.
            constexpr bool IROW = NBM <= 2 && 64 * E * NBM <= 128;
            if constexpr (IROW && CPNA == 0) {
                int bad = 0;
#pragma unroll
                for (int t = 0; t < NBM; ++t)
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int32_t w = cur[t][e];
                        bad |= (int)((unsigned)((int16_t)(w & 0xffff) + 2048) >= 4096u) |
                               (int)((unsigned)((w >> 16) + 2048) >= 4096u);
                    }
                wide = wide || __ballot(bad) != 0;
            }
            double qcf[E], qef[E], qcx, qex, qct, qet;
            if (IROW && !wide) {
                int pc[E], en[E];
#pragma unroll
                for (int e = 0; e < E; ++e) { pc[e] = 0; en[e] = 0; }
#pragma unroll
                for (int t = 0; t < NBM; ++t) {
                    if (t < nb_) {
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int32_t d = hx(t, xsl, e);
                            const int xr = (int16_t)(cur[t][e] & 0xffff), xi = cur[t][e] >> 16;
                            pc[e] += (int16_t)(d & 0xffff) * xr + (d >> 16) * xi;   // minn_rtl.py:616, exact
                            en[e] += xr * xr + xi * xi;                               // :617
                            hx(t, xsl, e) = cur[t][e];
                        }
                    }
                }
                RowPrefixI<E> ic, ie;
                ic.run(pc); ie.run(en);
#pragma unroll
                for (int e = 0; e < E; ++e) { qcf[e] = (double)ic.f[e]; qef[e] = (double)ie.f[e]; }
                qcx = (double)ic.excl; qex = (double)ie.excl; qct = (double)ic.tot; qet = (double)ie.tot;
            } else {
                double pc[E], en[E];
#pragma unroll
                for (int e = 0; e < E; ++e) { pc[e] = 0.0; en[e] = 0.0; }
#pragma unroll
                for (int t = 0; t < NBM; ++t) {
                    if (t < nb_) {
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int32_t d = hx(t, xsl, e);
                            const double xr = w_re(cur[t][e]), xi = w_im(cur[t][e]);
                            pc[e] += w_re(d) * xr + w_im(d) * xi;            // minn_rtl.py:616, exact
                            en[e] += xr * xr + xi * xi;                       // :617
                            hx(t, xsl, e) = cur[t][e];
                        }
                    }
                }
                RowPrefix<E> dc, de;
                dc.run(pc); de.run(en);
#pragma unroll
                for (int e = 0; e < E; ++e) { qcf[e] = dc.f[e]; qef[e] = de.f[e]; }
                qcx = dc.excl; qex = de.excl; qct = dc.tot; qet = de.tot;
            }
            const int s0r = k % NR;                                        // slot of row k
            const int s1 = (k + NR - MW) % NR, s2 = (k + NR - 2 * MW) % NR, s3 = (k + NR - 3 * MW) % NR;
            // steady rows (every lag row exists, every sample past the fill phase and inside the stream:
            // wave-uniform): no availability selects, no store guards - the same values
            if (k >= 3 * MW && (int64_t)RL * (k + 1) <= T) {
                const bool w_cp = a.corr_positive != nullptr, w_es = a.energy_scaled != nullptr, w_mv = a.mvalid != nullptr;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const double c0 = (CC + qcx) + qcf[e];
                    const double e0 = (CE + qex) + qef[e];
                    hac(s0r, e) = c0;
                    hae(s0r, e) = e0;
                    const double c1 = hac(s1, e), c2 = hac(s2, e);
                    const double e1 = hae(s1, e), e2 = hae(s2, e), e3 = hae(s3, e);
                    const double ct = 0.0 + ((c0 - c1) + (c1 - c2));       // minn_rtl.py:696
                    const double et = 0.0 + (((e0 - e1) + (e1 - e2)) + (e2 - e3));   // :697-701
                    const double cpos = ct > 0.0 ? ct : 0.0;               // :704
                    const double es = (a.thr_value == 0.0) ? 0.0 : et * a.thr_value;   // :718-721
                    const int i = nb + e;
                    const int li = (int)(i - s0);
                    hcp[seg_at(li)] = cpos;
                    hes[seg_at(li)] = es;
                    const int64_t gi = row_off + i;
                    a.corr_total[gi] = ct;
                    if (w_cp) a.corr_positive[gi] = cpos;
                    a.energy_total[gi] = et;
                    if (w_es) a.energy_scaled[gi] = es;
                    if (w_mv) a.mvalid[gi] = (uint8_t)(i >= vstart);
                }
                CC += qct; CE += qet;
                continue;
            }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const double c0 = (CC + qcx) + qcf[e];
                const double e0 = (CE + qex) + qef[e];
                hac(s0r, e) = c0;
                hae(s0r, e) = e0;
                // prefixes before the stream start are 0
                const double c1 = k >= MW ? hac(s1, e) : 0.0;
                const double c2 = k >= 2 * MW ? hac(s2, e) : 0.0;
                const double e1 = k >= MW ? hae(s1, e) : 0.0;
                const double e2 = k >= 2 * MW ? hae(s2, e) : 0.0;
                const double e3 = k >= 3 * MW ? hae(s3, e) : 0.0;
                const int i = nb + e;
                const double cr_ = (i >= Q - 1) ? c0 - c1 : 0.0;
                const double cp_ = (i >= 2 * Q - 1) ? c1 - c2 : 0.0;
                const double er_ = (i >= Q - 1) ? e0 - e1 : 0.0;
                const double ep_ = (i >= 2 * Q - 1) ? e1 - e2 : 0.0;
                const double ep2 = (i >= 3 * Q - 1) ? e2 - e3 : 0.0;
                const double ct = 0.0 + (cr_ + cp_);                       // minn_rtl.py:696
                const double et = 0.0 + ((er_ + ep_) + ep2);               // :697-701
                const double cpos = ct > 0.0 ? ct : 0.0;                   // :704
                const double es = (a.thr_value == 0.0) ? 0.0 : et * a.thr_value;   // :718-721
                const int li = (int)(i - s0);
                hcp[seg_at(li)] = cpos;
                hes[seg_at(li)] = es;
                if (i < T) {
                    const int64_t gi = row_off + i;
                    a.corr_total[gi] = ct;
                    if (a.corr_positive) a.corr_positive[gi] = cpos;
                    a.energy_total[gi] = et;
                    if (a.energy_scaled) a.energy_scaled[gi] = es;
                    if (a.mvalid) a.mvalid[gi] = (uint8_t)(i >= vstart);
                }
            }
            CC += qct; CE += qet;
        }
        if (!seq) continue;
        const int64_t c0 = s0 + (int64_t)SC * lane;                   // first sample of my chunk
        const int64_t send = min(T, s0 + SEG);
        bool abv[SC];
        double cp8[SC], own[SC];
        if (walk) {
            // ---------- phase B (RTL floor mode): one walker lane per stream of the workgroup -----
            // The integer floor-shift recursion does not merge nearby trajectories, so it runs as
            // written: wave 0, lane t walking stream t through the segment's corr_positive /
            // energy_scaled in LDS (rtl_walk).  The smoothed value goes back over energy_scaled
            // with the threshold decision in its sign bit (the state is never negative).
            lds_barrier();
            if (w == 0 && lane < wpb && (int64_t)blockIdx.x * wpb + lane < a.B) {
                const double* wcp = rsm + wave_dbl * lane + 2 * NR * E * 64;
                double* wes = const_cast<double*>(wcp) + SEG_PAD;
                const int n = (int)(send - s0);
                const int v0 = (int)max((int64_t)0, min((int64_t)n, (int64_t)vstart - s0));
                if (smode == 2) rtl_walk<2>(wcp, wes, n, v0, inv, scale, a.shift, sm, si);
                else if (smode == 1) rtl_walk<1>(wcp, wes, n, v0, inv, scale, a.shift, sm, si);
                else rtl_walk<0>(wcp, wes, n, v0, inv, scale, a.shift, sm, si);
            }
            lds_barrier();
#pragma unroll
            for (int e = 0; e < SC; ++e) {
                const int64_t p = c0 + e;
                const int at = seg_at(SC * lane + e);
                cp8[e] = hcp[at];
                const long long v = __double_as_longlong(hes[at]);
                own[e] = __longlong_as_double(v & 0x7fffffffffffffffll);
                abv[e] = p < T && v < 0;
            }
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // ---------- phase B (float IIR): segment-parallel, lane j = chunk j -----------------
            if (smode == 1) {                                          // shift 0: s = c (no chain)
#pragma unroll
                for (int e = 0; e < SC; ++e) {
                    const int64_t p = c0 + e;
                    own[e] = (p >= vstart && p < T) ? hcp[seg_at(SC * lane + e)] : 0.0;
                }
                // state holds where invalid (before vstart: the initial 0); positions >= T unused
                if (send - 1 >= vstart) sm = hcp[seg_at((int)(send - 1 - s0))];
            } else {
                // 1. chunk maps from s = 0: s_out = A·s_in + Z (approximate arithmetic is fine here)
                double A = 1.0, Z = 0.0;
                double cv[SC];
                bool upd[SC];
#pragma unroll
                for (int e = 0; e < SC; ++e) {
                    const int64_t p = c0 + e;
                    upd[e] = p >= vstart && p < T;
                    cv[e] = hcp[seg_at(SC * lane + e)];
                    if (upd[e]) {
                        Z = Z + (cv[e] - Z) * inv;
                        A = A * keep;
                    }
                }
                // inclusive wave scan of the affine maps (lane-1's map first, then mine): DPP
                // ladder row_shr 1/2/4/8, row_bcast 15/31
                double sa = A, sz = Z;
                const int rl = lane & 15;
                auto comb = [&](double pa, double pz, bool take) {
                    if (take) { sz = sa * pz + sz; sa = sa * pa; }
                };
                { const double pa = ofs::dpp_d<0x111>(sa), pz = ofs::dpp_d<0x111>(sz); comb(pa, pz, rl >= 1); }
                { const double pa = ofs::dpp_d<0x112>(sa), pz = ofs::dpp_d<0x112>(sz); comb(pa, pz, rl >= 2); }
                { const double pa = ofs::dpp_d<0x114>(sa), pz = ofs::dpp_d<0x114>(sz); comb(pa, pz, rl >= 4); }
                { const double pa = ofs::dpp_d<0x118>(sa), pz = ofs::dpp_d<0x118>(sz); comb(pa, pz, rl >= 8); }
                { const double pa = ofs::dpp_d<0x142>(sa), pz = ofs::dpp_d<0x142>(sz); comb(pa, pz, (lane & 31) >= 16); }
                { const double pa = ofs::dpp_d<0x143>(sa), pz = ofs::dpp_d<0x143>(sz); comb(pa, pz, lane >= 32); }
                // entering state of my chunk: exclusive map applied to the carried exact state
                const double ea = ofs::wave_shr1(sa, lane, 1.0), ez = ofs::wave_shr1(sz, lane, 0.0);
                double enter = lane == 0 ? sm : ea * sm + ez;
                // Interior segments (every sample updates) whose entering states are all 0 or >= 2^-700
                // run the step as fma(c - s, 2^-k, s): (c - s)·2^-k is exact (a power-of-two scaling that
                // cannot reach the subnormal range: s >= 0 shrinks by at most 2 per step, 256 steps per
                // segment, and a non-zero c - s is a multiple of ulp(s) >= 2^-752), so the fused add
                // rounds exactly as the reference's separate multiply and add do - 2 VALU per step
                // instead of 3 plus the per-sample update selects.  (States stay >= 2^-956 over the
                // segment, so |c - s| >= 2^-1008 when non-zero and the scaled value is normal for k <= 14.)
                const bool interior = s0 >= vstart && s0 + SEG <= T && a.shift <= 14;
                const bool fast = interior && __ballot(!(enter == 0.0 || enter >= 0x1p-700)) == 0;
                // 2./3. exact chunk runs until the chain is self-consistent: every lane runs the
                // reference recursion over its chunk from `enter`, then takes lane-1's leaving
                // state (DPP wave_shr:1) as its new `enter`; stop when no lane's entering state
                // changes.  Lane 0 starts exact, and after round r lanes 0..r are exact: <= 64 rounds.
#ifndef OFS_RTL_MAXROUNDS                   // diagnostic builds only: < 64 cuts the rounds (inexact)
#define OFS_RTL_MAXROUNDS 64
#endif
                // Fast segments test the chain every OFS_RTL_RPT-th round: an untested round's hand-over
                // and the tested round's are the same operation, and a consistent tested round is the
                // reference trajectory as before; the test (compare, ballot, scalar branch) is what the
                // group saves, at most RPT - 1 extra rounds per segment (RPT 1 / 2 / 3 / 4: cfg2b 0.048
                // / 0.043 / 0.0414 / 0.0413 ms, profiles/r04t_*).
#ifndef OFS_RTL_RPT
#define OFS_RTL_RPT 4                      // rounds per consistency test on fast segments (tuning builds)
#endif
                if (fast) {
                    for (int round = 0; round <= OFS_RTL_MAXROUNDS; round += OFS_RTL_RPT) {
                        double st = enter;
#pragma unroll
                        for (int r = 1; r < OFS_RTL_RPT; ++r) {            // untested rounds
#pragma unroll
                            for (int e = 0; e < SC; ++e) st = fma(cv[e] - st, inv, st);
                            enter = ofs::wave_shr1(st, lane, sm);
                            st = enter;
                        }
#pragma unroll
                        for (int e = 0; e < SC; ++e) {
                            st = fma(cv[e] - st, inv, st);
                            own[e] = st;
                        }
                        const double prev_leave = ofs::wave_shr1(st, lane, sm);
#if OFS_RTL_ROUNDS_DEBUG
                        dbg_rounds += OFS_RTL_RPT;
#endif
                        if (__ballot(!same_bits(enter, prev_leave)) == 0) {
                            sm = readlane(st, 63);
                            break;
                        }
                        enter = prev_leave;
                    }
                } else {
                    for (int round = 0; round <= OFS_RTL_MAXROUNDS; ++round) {
                        double st = enter;
#pragma unroll
                        for (int e = 0; e < SC; ++e) {
                            if (upd[e]) st = st + (cv[e] - st) * inv;
                            own[e] = st;
                        }
                        const double prev_leave = ofs::wave_shr1(st, lane, sm);
#if OFS_RTL_ROUNDS_DEBUG
                        ++dbg_rounds;
#endif
                        if (__ballot(!same_bits(enter, prev_leave)) == 0) {
                            sm = readlane(st, 63);
                            break;
                        }
                        enter = prev_leave;
                    }
                }
            }
            // ---------- phase C: threshold (chunk layout) -----------------------------------------
#pragma unroll
            for (int e = 0; e < SC; ++e) {
                const int64_t p = c0 + e;
                const int at = seg_at(SC * lane + e);
                cp8[e] = hcp[at];
                abv[e] = p >= vstart && p < T && (own[e] * scale >= hes[at]);      // minn_rtl.py:717-722
            }
        }
        // ---------- phase C: gate; the chunk's stores wait for the next segment's row take -----------
        pend = true;
        pend_c0 = c0;
#pragma unroll
        for (int e = 0; e < SC; ++e) { pend_own[e] = own[e]; pend_abv[e] = abv[e]; }
        if (a.detect && send > vstart) {
            double none[SC];
#pragma unroll
            for (int e = 0; e < SC; ++e) none[e] = 0.0;
            gate.row_flags(lane, g, (int)c0, (int)T, abv, cp8, none, none, none);
        }
        __builtin_amdgcn_wave_barrier();                               // LDS reuse by the next segment
    }
    if (pend) store_chunk(pend_c0, pend_own, pend_abv);
    if (a.detect) gate.finish(lane, (int)T, a.n_ev + b, a.open_start ? a.open_start + b : nullptr);
#if OFS_RTL_ROUNDS_DEBUG                    // tools/rtl_rounds.py: speculation rounds over the stream
    __builtin_amdgcn_wave_barrier();
    if (a.open_start && lane == 0) a.open_start[b] = dbg_rounds;
#endif
}

// ---- dispatch -------------------------------------------------------------------------------
bool exact_enabled() {                  // variant EXACT=0 forces the general engine (A/B, tests)
    return !ofs::variant_off(ofs::V_EXACT);
}

template <int E, int MR, int NA>
int aa_launch(int fmt, const AaFastArgs& a, hipStream_t st) {
    if (fmt == OFS_C128)
        hipLaunchKernelGGL((aa_exact_kernel<OFS_C128, E, MR, NA>), dim3((unsigned)((a.B + xa_wg(OFS_C128, MR, NA) / 64 - 1) / (xa_wg(OFS_C128, MR, NA) / 64))), dim3(xa_wg(OFS_C128, MR, NA)), ofs::occ_lds(), st, a);
    else if (fmt == OFS_CP12)
        hipLaunchKernelGGL((aa_exact_kernel<OFS_CP12, E, MR, NA>), dim3((unsigned)((a.B + xa_wg(OFS_CP12, MR, NA) / 64 - 1) / (xa_wg(OFS_CP12, MR, NA) / 64))), dim3(xa_wg(OFS_CP12, MR, NA)), ofs::occ_lds(), st, a);
    else
        hipLaunchKernelGGL((aa_exact_kernel<OFS_CI16, E, MR, NA>), dim3((unsigned)((a.B + xa_wg(OFS_CI16, MR, NA) / 64 - 1) / (xa_wg(OFS_CI16, MR, NA) / 64))), dim3(xa_wg(OFS_CI16, MR, NA)), ofs::occ_lds(), st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}
template <int E, int MR>
int aa_launch_na(int fmt, int na, const AaFastArgs& a, hipStream_t st) {
    switch (na) {
        case 1: return aa_launch<E, MR, 1>(fmt, a, st);
        case 2: return aa_launch<E, MR, 2>(fmt, a, st);
    }
    return 0;
}
template <int E>
int aa_launch_mr(int fmt, int mr, int na, const AaFastArgs& a, hipStream_t st) {
    switch (mr) {
        case 1: return aa_launch_na<E, 1>(fmt, na, a, st);
        case 2: return aa_launch_na<E, 2>(fmt, na, a, st);
        case 4: return aa_launch_na<E, 4>(fmt, na, a, st);
        case 8: return aa_launch_na<E, 8>(fmt, na, a, st);
    }
    return 0;
}

template <int E, int MW, int CPNA, int NBM>
int rtl_launch_k(const RtlExactArgs& a, hipStream_t st) {
    const size_t per_wave = rtl_wave_lds(E, MW, a.nb);
    int wpb = 4;                                             // waves (streams) per workgroup
    const int64_t wv = ofs::variant(ofs::V_RTL_WPB);        // tuning: 1, 2 or 4
    if (wv == 1 || wv == 2) wpb = (int)wv;
    while (wpb > 1 && per_wave * wpb > 64 * 1024) wpb >>= 1;
    const size_t lds = per_wave * wpb + ofs::occ_lds();
    auto k = rtl_exact_kernel<E, MW, CPNA, NBM>;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return OFS_EHIP;
    hipLaunchKernelGGL(k, dim3((unsigned)((a.B + wpb - 1) / wpb)), dim3(64 * wpb), lds, st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

template <int E, int MW>
int rtl_launch(int fmt, const RtlExactArgs& a, hipStream_t st) {
    if (fmt == OFS_CP12) return a.nb == 1 ? rtl_launch_k<E, MW, 1, 1>(a, st) : rtl_launch_k<E, MW, 2, 2>(a, st);
    return a.nb == 1 ? rtl_launch_k<E, MW, 0, 1>(a, st) : rtl_launch_k<E, MW, 0, 4>(a, st);
}

}  // namespace

// 10*E + MR of the wave-per-stream fp64 aa kernel for a shape (+100 for complex128 input), 0 if
// not covered
int ofs_aa_exact_plan(int fmt, int precision, int n_ant, int64_t T, int L) {
    if ((fmt != OFS_CI16 && fmt != OFS_C128 && fmt != OFS_CP12) || precision != OFS_FP64 || n_ant < 1 || n_ant > 2 ||
        (!exact_enabled() && fmt != OFS_CP12))
        return 0;
    if ((fmt == OFS_CI16 || fmt == OFS_CP12) && (T < 1 || T * n_ant > (1 << 21) || T > 0x7fffffff / 2))
        return 0;                                                // sums < 2^53
    // complex128: stream-wide fp64 prefix differences.  Their error, O(eps·|prefix|) <=
    // O(eps·n·max term), is of the same order as the reference's own recursive running sum
    // (sum = sum + new - oldest, sync_aa.py:331-342, which accumulates O(eps·n·max term)), so
    // any stream length keeps the reference's error regime (checked on the T = 5315, 2-antenna
    // grid goldens and against the general engine's tiles)
    if (fmt == OFS_C128 && (T < 1 || T > 0x3fffffff)) return 0;
    if (fmt == OFS_C128 && n_ant == 2 && L > 512) return 0;  // fp64 rings of 2 x 1024 lags spill
    const int f = fmt == OFS_C128 ? 100 : 0;
    if (L == 64) return f + 11;
    if (L % 128 == 0 && (L == 128 || L == 256 || L == 512 || L == 1024)) return f + 20 + L / 128;
    return 0;
}

int ofs_aa_exact_try(int fmt, int precision, int n_ant, const AaFastArgs& a, hipStream_t st) {
    const int plan = ofs_aa_exact_plan(fmt, precision, n_ant, a.T, a.L);
    if (!plan) return 0;
    const int E = (plan % 100) / 10, mr = plan % 10;
    if (E == 1) return aa_launch_na<1, 1>(fmt, n_ant, a, st);
    return aa_launch_mr<2>(fmt, mr, n_ant, a, st);
}

int ofs_rtl_exact_plan(int fmt, int n_br, int64_t T, int Q) {
    if (fmt == OFS_CP12 ? (n_br < 1 || n_br > 2) : (fmt != OFS_CI16 || n_br < 1 || n_br > 4 || !exact_enabled()))
        return 0;
    if (T < 1 || T * n_br > (1 << 21)) return 0;
    for (int e : {1, 2, 4}) {
        if (Q % (64 * e)) continue;
        const int mw = Q / (64 * e);
        if (mw == 1 || mw == 2) return 10 * e + mw;
    }
    return 0;                                                // Q > 512 or not a multiple of 64
}

int ofs_rtl_exact_try(int fmt, int n_br, const RtlExactCall& c, hipStream_t st) {
    const int plan = ofs_rtl_exact_plan(fmt, n_br, c.T, c.Q);
    if (!plan) return 0;
    RtlExactArgs a;
    a.x = c.x; a.B = c.B; a.T = c.T; a.nb = n_br; a.Q = c.Q;
    a.shift = c.shift; a.smooth_mode = c.smooth_mode; a.frac_bits = c.frac_bits; a.thr_value = c.thr_value;
    a.corr_total = c.corr_total; a.corr_positive = c.corr_positive; a.smooth = c.smooth;
    a.energy_total = c.energy_total; a.corr_scaled = c.corr_scaled; a.energy_scaled = c.energy_scaled;
    a.mvalid = c.mvalid; a.above = c.above; a.detect = c.detect; a.hyst = c.hyst; a.toff = c.toff;
    a.max_ev = c.max_ev; a.n_ev = c.n_ev; a.ev = c.ev; a.open_start = c.open_start;

    switch (plan) {
        case 11: return rtl_launch<1, 1>(fmt, a, st);
        case 12: return rtl_launch<1, 2>(fmt, a, st);
        case 21: return rtl_launch<2, 1>(fmt, a, st);
        case 22: return rtl_launch<2, 2>(fmt, a, st);
        case 41: return rtl_launch<4, 1>(fmt, a, st);
        case 42: return rtl_launch<4, 2>(fmt, a, st);
    }
    return 0;
}
