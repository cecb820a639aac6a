// backend.hip — batched OFDM receiver back-end behind the timing/CFO path (core.py:171-176,
// :179-196, :339-370, :443-469 as chained by sc.run_simulation, sc.py:274-311):
//
//   cfo      = estimate_cfo_from_cp(rx, pilot_start, N, cp, fs)        (or given per frame)
//   rx_eff   = mean_br( apply_cfo(rx, -cfo, fs) )                       (core.py:123-138)
//   y_pilot  = ofdm_fft_used(rx_eff[pilot_start + cp : + N])            (core.py:171-176)
//   h        = ls_channel_estimate(y_pilot, pilot_used)                  (core.py:339-341)
//   slope, sto = estimate_timing_offset_from_phase_slope(h)             (core.py:443-469)
//   y_data   = ofdm_fft_used(rx_eff[data_start + cp : + N])
//   xhat     = equalize(y_data, h)                                       (core.py:344-345)
//   xa, gain = align_complex_gain(xhat, data_used)                      (core.py:357-362)
//   evm, db  = evm_rms_db(xa, data_used)                                 (core.py:365-370)
//
// One 256-thread workgroup per frame, fp64 throughout (the reference is float64):
//   * the two N-point DFTs are iterative radix-2 FFTs in LDS (bit-reversed load, twiddles
//     from sincospi of exact rationals, one table per workgroup), N a power of two <= 4096;
//   * fftshift + used-bin gather collapse to X[k mod N] for the centred bin indices k;
//   * np.unwrap is a per-bin correction (numpy's mod / boundary rule) followed by a prefix sum
//     (block scan), the phase-slope fit and all means are block reductions.
// Per-frame, O(N log N) work: compute-bound and tiny next to the metric kernels.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <math.h>
#include <stdint.h>
#include "ofdmsync.h"
#include "ofs_common.h"
#include "be_math.h"

namespace {

#ifndef OFS_BE_WG
#define OFS_BE_WG 256
#endif
constexpr int BW = OFS_BE_WG;     // threads per frame workgroup
constexpr int BNMAX = 4096;

struct BeArgs {
    int fmt; const void* x; int64_t B, T; int nb; int N, cp, n_used; double fs;
    const int64_t* pilot_start; const int64_t* data_start; const double* cfo_in;
    const int32_t* bins; const double2* pilot; int64_t pilot_stride; const double2* data; int64_t data_stride;
    double* cfo_out; double2* h_out; double2* xa_out; double2* gain_out; double* evm_out; double* evm_db_out;
    double* slope_out; double* sto_out;
};

template <int FMT>
__device__ __forceinline__ double2 ld(const void* p, int64_t i) {
    if constexpr (FMT == OFS_C64) {
        const float2 v = static_cast<const float2*>(p)[i];
        return make_double2(v.x, v.y);
    } else if constexpr (FMT == OFS_C128) {
        return static_cast<const double2*>(p)[i];
    } else {
        const short2 v = static_cast<const short2*>(p)[i];
        return make_double2(v.x, v.y);
    }
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// a / b exactly as numpy divides complex128 (Smith's algorithm with the reciprocal scale
// scl = 1 / (b.x + b.y * rat), no contraction): bit-identical to numpy on the same operands
#ifndef OFS_BE_CDIV_SEL
#define OFS_BE_CDIV_SEL 1          // 0: numpy's two branches as branches (A/B)
#endif
__device__ __forceinline__ double2 cdiv(double2 a, double2 b) {
#pragma clang fp contract(off)
    const double br = fabs(b.x), bi = fabs(b.y);
#if OFS_BE_CDIV_SEL
    // Branch-free: both of numpy's cases are one formula on swapped operands (the larger |b|
    // component p, the other q; a's components u, v in the same order), so a wave whose lanes
    // split between the cases runs ONE pair of fp64 divisions instead of both branches' pairs.
    // Bit-identical: case 2's real part a.x·rat + a.y = u + v·rat (addition commutes exactly) and
    // its imaginary part a.y·rat - a.x = -(v - u·rat) (x - y = -(y - x) exactly, then ·scl).
    // b = 0: numpy's a.x / |b.x|, a.y / |b.y| = a·(+inf) (signed inf, or NaN for a 0 or NaN part).
    const bool c1 = br >= bi;
    const double p = c1 ? b.x : b.y, q = c1 ? b.y : b.x;
    const double u = c1 ? a.x : a.y, v = c1 ? a.y : a.x;
    const double rat = q / p, scl = 1.0 / (p + q * rat);
    const double re = (u + v * rat) * scl, t = (v - u * rat) * scl;
    const bool zero = br == 0.0 && bi == 0.0;
    return make_double2(zero ? a.x * __builtin_inf() : re, zero ? a.y * __builtin_inf() : (c1 ? t : -t));
#else
    if (br >= bi) {
        if (br == 0.0 && bi == 0.0) return make_double2(a.x / br, a.y / bi);
        const double rat = b.y / b.x, scl = 1.0 / (b.x + b.y * rat);
        return make_double2((a.x + a.y * rat) * scl, (a.y - a.x * rat) * scl);
    }
    const double rat = b.x / b.y, scl = 1.0 / (b.y + b.x * rat);
    return make_double2((a.x * rat + a.y) * scl, (a.y * rat - a.x) * scl);
#endif
}

// workgroup barrier ordering LDS only: every barrier here orders LDS traffic (the global inputs
// are read-only and outputs are never read back), and a __syncthreads() fence would also wait
// for the frame's output stores in flight (vmcnt(0)) at each of the ~45 barriers of a frame
// (measured neutral here, r02aw: the frame's stores are few)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// block-wide sum of doubles (all threads get the result)
__device__ double block_sum(double v, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    lds_barrier();
    if (lane == 0) red[w] = v;
    lds_barrier();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < BW / 64; ++k) s += red[k];
    return s;
}

// numpy.mod for float64 (result has the sign of the divisor)
__device__ __forceinline__ double np_mod(double a, double b) {
    // fmod(a, b) = a - n·b exactly; for b > 0 and |a| < 2b, n is 0 or ±1 and a ∓ b is exact (Sterbenz:
    // |a| in [b, 2b]), so the library's general fmod (an iterative routine) is needed only beyond that -
    // the unwrap's a = dd + pi with |dd| <= 2 pi never goes there.  Same bits: a zero result takes the
    // sign of b below either way.
    double m;
    if (b > 0.0 && fabs(a) < 2.0 * b) m = a >= b ? a - b : (a <= -b ? a + b : a);
    else m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0.0) != (m < 0.0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

// N-point forward DFT of buf (bit-reversed in, natural order out) in LDS; tw[j] = exp(-2 pi i j / N).
// Iterative radix-2 DIT, two stages fused per pass: a thread takes the four elements p, p+h,
// p+2h, p+3h of a 4h-group and applies the len-2h butterflies then the len-4h ones in registers -
// the same operations in the same order as two radix-2 passes (bit-identical), half the passes,
// barriers and LDS round trips.  An odd stage count starts with one radix-2 pass.
__device__ void fft_lds(double2* buf, const double2* tw, int N, int LB) {
    int len = 2;
    if (LB & 1) {                                            // len-2 stage alone (w = 1)
        for (int j = threadIdx.x; j < N / 2; j += BW) {
            const double2 u = buf[2 * j], v = buf[2 * j + 1];
            const double2 t = cmul(tw[0], v);
            buf[2 * j] = make_double2(u.x + t.x, u.y + t.y);
            buf[2 * j + 1] = make_double2(u.x - t.x, u.y - t.y);
        }
        lds_barrier();
        len = 4;
    }
    for (; len <= N; len <<= 2) {                            // stages len (h = len/2) and 2*len
        const int h = len >> 1;
        const int s1 = N / len, s2 = N / (2 * len);          // twiddle strides of the two stages
        for (int j = threadIdx.x; j < N / 4; j += BW) {
            const int g = j / h, k = j - g * h;
            const int p = g * 4 * h + k;
            const double2 a0 = buf[p], a1 = buf[p + h], a2 = buf[p + 2 * h], a3 = buf[p + 3 * h];
            const double2 w1 = tw[k * s1];
            const double2 t1 = cmul(w1, a1), t3 = cmul(w1, a3);
            const double2 b0 = make_double2(a0.x + t1.x, a0.y + t1.y), b1 = make_double2(a0.x - t1.x, a0.y - t1.y);
            const double2 b2 = make_double2(a2.x + t3.x, a2.y + t3.y), b3 = make_double2(a2.x - t3.x, a2.y - t3.y);
            const double2 u = cmul(tw[k * s2], b2), v = cmul(tw[(k + h) * s2], b3);
            buf[p] = make_double2(b0.x + u.x, b0.y + u.y);
            buf[p + 2 * h] = make_double2(b0.x - u.x, b0.y - u.y);
            buf[p + h] = make_double2(b1.x + v.x, b1.y + v.y);
            buf[p + 3 * h] = make_double2(b1.x - v.x, b1.y - v.y);
        }
        lds_barrier();
    }
}

// estimate_timing_offset_from_phase_slope (core.py:443-469) on ph[0..U) = angle(h) in LDS (all
// threads): np.unwrap restated as per-bin corrections (numpy's float mod and boundary rule) and
// an exclusive block scan - ph becomes the unwrapped phase - then the LS slope over the abscissa
// bins[u].  Ends with the workgroup converged (block_sum).
__device__ double unwrap_slope(double* ph, const int32_t* bins, int U, double* red, double* scan_tot) {
    {
        // each thread owns a contiguous run of bins; correction[u] applies to bins >= u
        const int per = (U + BW - 1) / BW;
        const int u0 = threadIdx.x * per, u1 = min(U, u0 + per);
        double local = 0.0;
        for (int u = max(u0, 1); u < u1; ++u) {
            const double dd = ph[u] - ph[u - 1];
            if (!(fabs(dd) < M_PI)) {                        // numpy's correction only where |dd| >= pi
                double dm = np_mod(dd + M_PI, 2.0 * M_PI) - M_PI;
                if (dm == -M_PI && dd > 0.0) dm = M_PI;
                local += dm - dd;
            }
        }
        // exclusive block scan of the per-thread totals
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        double incl = local;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
        }
        if (lane == 63) scan_tot[w] = incl;
        lds_barrier();
        double base = incl - local;
        for (int k = 0; k < w; ++k) base += scan_tot[k];
        lds_barrier();
        // rewrite ph[u] = unwrapped phase (reads of ph[u-1] done above, before the barrier)
        double run = base, prev_raw = u0 >= 1 && u0 < U ? ph[u0 - 1] : 0.0;
        lds_barrier();
        for (int u = u0; u < u1; ++u) {
            const double raw = ph[u];
            if (u >= 1) {
                const double dd = raw - prev_raw;
                if (!(fabs(dd) < M_PI)) {
                    double dm = np_mod(dd + M_PI, 2.0 * M_PI) - M_PI;
                    if (dm == -M_PI && dd > 0.0) dm = M_PI;
                    run += dm - dd;
                }
            }
            prev_raw = raw;
            ph[u] = raw + run;
        }
        lds_barrier();
    }
    double sk = 0.0, sp = 0.0;
    for (int u = threadIdx.x; u < U; u += BW) { sk += (double)bins[u]; sp += ph[u]; }
    const double kmean = block_sum(sk, red) / (double)U;
    const double pmean = block_sum(sp, red) / (double)U;
    double skk = 0.0, skp = 0.0;
    for (int u = threadIdx.x; u < U; u += BW) {
        const double kz = (double)bins[u] - kmean, pz = ph[u] - pmean;
        skk += kz * kz; skp += kz * pz;
    }
    const double den = block_sum(skk, red) + 1e-12;
    return block_sum(skp, red) / den;
}

__device__ __forceinline__ int bitrev(int v, int bits) { return (int)(__brev((unsigned)v) >> (32 - bits)); }

// load rx_eff[s : s + N] = mean_br(rx[br] * exp(-i 2 pi cfo n / fs)) bit-reversed into buf.  The
// tone of a thread's samples n = tid + BW·m comes from one sincos at its first sample and a
// rotation by exp(i·phase(BW)) per step (angle addition: <= N/BW steps, ~1e-15 relative)
template <int FMT>
__device__ void load_window(const BeArgs& a, int64_t b, int64_t s, double cfo, double2* buf, int LB) {
    const double w0 = 2.0 * M_PI * (-cfo);
    double sn, cs, ss, cc;
    sincos(w0 * (double)(s + (int64_t)threadIdx.x) / a.fs, &sn, &cs);   // core.apply_cfo's phase
    sincos(w0 * (double)BW / a.fs, &ss, &cc);
    double2 tone = make_double2(cs, sn);
    const double2 step = make_double2(cc, ss);
    for (int n = threadIdx.x; n < a.N; n += BW) {
        const int64_t i = s + n;
        double2 acc = make_double2(0.0, 0.0);
        if (i >= 0 && i < a.T) {
            for (int br = 0; br < a.nb; ++br) {
                const double2 v = cmul(ld<FMT>(a.x, (b * a.nb + br) * a.T + i), tone);
                acc.x += v.x; acc.y += v.y;
            }
            acc.x /= (double)a.nb; acc.y /= (double)a.nb;              // np.mean over branches
        }
        buf[bitrev(n, LB)] = acc;
        tone = cmul(tone, step);
    }
    lds_barrier();
}

// the thread index, opaque to the compiler inside the fast kernel's frame loop: values derived from
// it (addresses, masks, bin indices) are recomputed per frame instead of being hoisted out of the
// loop and held in registers across it (OFS_BE_REMAT = 0: plain threadIdx.x, A/B)
#ifndef OFS_BE_REMAT
#define OFS_BE_REMAT 1
#endif
__device__ __forceinline__ int be_tid() {
    int t = threadIdx.x;
#if OFS_BE_REMAT
    asm volatile("" : "+v"(t));
#endif
    return t;
}

// log10 for the per-frame EVM in dB (one lane per frame): out of line, so that ocml's coefficients
// are not hoisted out of the fast kernel's frame loop into registers held across it
__device__ __attribute__((noinline)) double be_log10(double x) { return log10(x); }

// the fast kernel's per-bin outputs (h, xa), streamed past the caches (nothing here reads them back):
// r05ax, bit-identical, 0.710 -> 0.702 ms (N 2048), 0.819 -> 0.815 (1024), 0.898 -> 0.890 (4096)
#ifndef OFS_BE_NT
#define OFS_BE_NT 1
#endif
typedef double be_d2v __attribute__((ext_vector_type(2)));
#ifndef OFS_BE_ST16
#define OFS_BE_ST16 1              // 0: two 8-byte halves per complex output (A/B)
#endif
__device__ __forceinline__ void be_st(double2* p, double2 v) {
#if OFS_BE_NT
#if OFS_BE_ST16
    __builtin_nontemporal_store(be_d2v{v.x, v.y}, reinterpret_cast<be_d2v*>(p));   // one 16-byte store
#else
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
#endif
#else
    *p = v;
#endif
}

template <int FMT> struct BeRaw { using T = float2; };          // the input word kept in registers
template <> struct BeRaw<OFS_C128> { using T = double2; };
template <> struct BeRaw<OFS_CI16> { using T = short2; };
template <int FMT>
__device__ __forceinline__ typename BeRaw<FMT>::T ld_raw(const void* p, int64_t i) {
    return static_cast<const typename BeRaw<FMT>::T*>(p)[i];
}
template <class T>
__device__ __forceinline__ double2 widen(T v) { return make_double2((double)v.x, (double)v.y); }
template <class T>
__device__ __forceinline__ T zero_raw() { T z; z.x = 0; z.y = 0; return z; }

constexpr int BE_CPT = 2;                     // CP samples per thread (cp <= 2·BW on the fast path)

// one window of NBT branches, SPT samples per thread, raw words.  A window wholly inside [0, T)
// (the usual case, one wave-uniform test) loads without per-element guards, from one base pointer
// per branch, so the loads need no per-element 64-bit address or condition registers.
template <int FMT, int SPT, int NBT>
struct BeWindow {
    typename BeRaw<FMT>::T v[NBT][SPT];
    __device__ __forceinline__ void issue(const BeArgs& a, int64_t b, int64_t s) {
        using T = typename BeRaw<FMT>::T;
        const T* x = static_cast<const T*>(a.x);
        if (s >= 0 && s + SPT * BW <= a.T) {
#pragma unroll
            for (int r = 0; r < NBT; ++r) {
                const T* p = x + (b * NBT + r) * a.T + s + be_tid();
#pragma unroll
                for (int m = 0; m < SPT; ++m) v[r][m] = p[BW * m];
            }
        } else {
#pragma unroll
            for (int r = 0; r < NBT; ++r)
#pragma unroll
                for (int m = 0; m < SPT; ++m) {
                    const int64_t i = s + be_tid() + BW * m;
                    v[r][m] = (i >= 0 && i < a.T) ? x[(b * NBT + r) * a.T + i] : zero_raw<T>();
                }
        }
    }
};
// the CP correlation's samples x[ps + n], x[ps + N + n], n = tid + BW·m < cp
template <int FMT, int NBT>
struct BeCp {
    typename BeRaw<FMT>::T u[NBT][BE_CPT], w[NBT][BE_CPT];
    __device__ __forceinline__ void issue(const BeArgs& a, int64_t b, int64_t ps) {
        using T = typename BeRaw<FMT>::T;
        const T* x = static_cast<const T*>(a.x);
        const bool full = ps >= 0 && ps + a.N + a.cp <= a.T;
#pragma unroll
        for (int r = 0; r < NBT; ++r) {
            const T* p = x + (b * NBT + r) * a.T + ps + be_tid();
#pragma unroll
            for (int m = 0; m < BE_CPT; ++m) {
                const int n = be_tid() + BW * m;
                const int64_t i0 = ps + n, i1 = ps + a.N + n;
                const bool ok = !a.cfo_in && n < a.cp && (full || (i0 >= 0 && i1 < a.T));
                u[r][m] = ok ? p[BW * m] : zero_raw<T>();
                w[r][m] = ok ? p[a.N + BW * m] : zero_raw<T>();
            }
        }
    }
};

// window (registers) -> rx_eff = mean_br(x · exp(-i 2 pi cfo n / fs)) bit-reversed into buf
template <int FMT, int SPT, int NBT>
__device__ __forceinline__ void place_window(const BeArgs& a, int64_t s, double cfo, const BeWindow<FMT, SPT, NBT>& win,
                                             double2* buf, int LB) {
    const double w0 = 2.0 * M_PI * (-cfo);
    double sn, cs, ss, cc;
    ofs_bemath::sincos_lean(w0 * (double)(s + (int64_t)be_tid()) / a.fs, &sn, &cs);   // core.apply_cfo's phase
    ofs_bemath::sincos_lean(w0 * (double)BW / a.fs, &ss, &cc);
    double2 tone = make_double2(cs, sn);
    const double2 step = make_double2(cc, ss);
    const int rb = bitrev(be_tid(), LB);
#pragma unroll
    for (int m = 0; m < SPT; ++m) {
        const int n = be_tid() + BW * m;
        const int64_t i = s + n;
        double2 acc = make_double2(0.0, 0.0);
        if (i >= 0 && i < a.T) {
#pragma unroll
            for (int r = 0; r < NBT; ++r) {
                const double2 w = cmul(widen(win.v[r][m]), tone);
                acc.x += w.x; acc.y += w.y;
            }
            acc.x /= (double)NBT; acc.y /= (double)NBT;                 // np.mean over branches
        }
        buf[rb + bitrev(BW * m, LB)] = acc;                           // bit sets of tid and BW·m disjoint
        tone = cmul(tone, step);
    }
    lds_barrier();
}

// ---- fast path: N = SPT·BW, NBT branches, cp <= 2·BW, n_used <= UPT·BW (compile time) ---------
// Against the generic kernel below (r03q/r03r: a frame waited ~40 % of its time on serialized
// HBM round trips, and its 77 KB of LDS held the CU at 2 workgroups):
//  * each window's nb·SPT loads per thread (and the CP correlation's) are issued together into
//    registers (raw input words) before the first is used: one round trip per window;
//  * the channel estimate h and the equalised xhat never leave registers: thread t owns the used
//    bins u = t + BW·j in the LS, EQ and EVM loops alike, so only the phases (unwrap: cross-bin)
//    go to LDS;
//  * the twiddle table holds N/4 entries (w^{j+N/4} = -i·w^j);
// so a workgroup needs N·16 + N/4·16 bytes of LDS (40 KB at N = 2048, the phases and reduction
// slots overlaying the sample buffer: OFS_BE_LDS40) and, with be_math.h's lean atan2 / sincos,
// 128 VGPRs: 4 workgroups (16 waves) per CU.
// variant BE_FAST=0 selects the generic kernel (A/B).
#ifndef OFS_BE_TIMING
#define OFS_BE_TIMING 0            // diagnostic builds: per-phase cycles (tools/be_phase.py)
#endif
#if OFS_BE_TIMING
__device__ unsigned long long be_prof[12];
#define BE_T(i)                                                                                      \
    if (threadIdx.x == 0) { const long long t_ = __builtin_amdgcn_s_memtime(); tacc[i] += t_ - tprev; tprev = t_; }
#else
#define BE_T(i)
#endif

__device__ __forceinline__ double2 twq_at(const double2* twq, int j, int Q) {
    if (j < Q) return twq[j];
    const double2 v = twq[j - Q];
    return make_double2(v.y, -v.x);                          // w^{j} = -i·w^{j-N/4}
}

// fft_lds with the quarter twiddle table (same butterflies, same order)
__device__ void fft_lds_q(double2* buf, const double2* twq, int N, int LB) {
    const int Q = N / 4;
    int len = 2;
    if (LB & 1) {
        for (int j = threadIdx.x; j < N / 2; j += BW) {
            const double2 u = buf[2 * j], v = buf[2 * j + 1];
            const double2 t = cmul(twq[0], v);
            buf[2 * j] = make_double2(u.x + t.x, u.y + t.y);
            buf[2 * j + 1] = make_double2(u.x - t.x, u.y - t.y);
        }
        lds_barrier();
        len = 4;
    }
    for (; len <= N; len <<= 2) {
        const int h = len >> 1;
        const int s1 = N / len, s2 = N / (2 * len);
        for (int j = threadIdx.x; j < N / 4; j += BW) {
            const int g = j / h, k = j - g * h;
            const int p = g * 4 * h + k;
            const double2 a0 = buf[p], a1 = buf[p + h], a2 = buf[p + 2 * h], a3 = buf[p + 3 * h];
            const double2 w1 = twq_at(twq, k * s1, Q);
            const double2 t1 = cmul(w1, a1), t3 = cmul(w1, a3);
            const double2 b0 = make_double2(a0.x + t1.x, a0.y + t1.y), b1 = make_double2(a0.x - t1.x, a0.y - t1.y);
            const double2 b2 = make_double2(a2.x + t3.x, a2.y + t3.y), b3 = make_double2(a2.x - t3.x, a2.y - t3.y);
            const double2 u = cmul(twq_at(twq, k * s2, Q), b2), v = cmul(twq_at(twq, (k + h) * s2, Q), b3);
            buf[p] = make_double2(b0.x + u.x, b0.y + u.y);
            buf[p + 2 * h] = make_double2(b0.x - u.x, b0.y - u.y);
            buf[p + h] = make_double2(b1.x + v.x, b1.y + v.y);
            buf[p + 3 * h] = make_double2(b1.x - v.x, b1.y - v.y);
        }
        lds_barrier();
    }
}

#ifndef OFS_BE_RED2
#define OFS_BE_RED2 1              // fast kernel: block sums alternate between two slot sets, one barrier each
#endif
#ifndef OFS_BE_ZSCAN
#define OFS_BE_ZSCAN 1             // block sums by the zero-filled DPP ladder (0: predicated ladder, A/B)
#endif
// NV block-wide sums with one pair of barriers: DPP wave sums (inclusive scan, lane 63), then the
// BW/64 wave totals through LDS; every thread gets the NV results.
template <int NV, bool SYNC = false>
__device__ __forceinline__ void block_sums(double (&v)[NV], double* red) {
    const int lane = be_tid() & 63, w = be_tid() >> 6;
#if OFS_BE_ZSCAN
    // zero-filled DPP ladder (no lane predicates; the same additions in the same order), the wave
    // total written by lane 63 itself (no readlane)
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = ofs::scan_add(v[i]);
    if (!OFS_BE_RED2 || SYNC) lds_barrier();                 // red's previous readers are done (RED2:
                                                             // alternating slots, the previous call's
                                                             // barrier orders them; SYNC: the slots
                                                             // overlay LDS data other waves may still read)
    if (lane == 63)
#pragma unroll
        for (int i = 0; i < NV; ++i) red[w * NV + i] = v[i];
#else
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = ofs::readlane(ofs::wave_scan_add(v[i], lane), 63);
    lds_barrier();                                           // red's previous readers are done
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) red[w * NV + i] = v[i];
#endif
    lds_barrier();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < BW / 64; ++k) t += red[k * NV + i];
        v[i] = t;
    }
}

// estimate_timing_offset_from_phase_slope (core.py:443-469) on ph[0..U) = angle(h) in LDS, with the
// frame-invariant bin statistics precomputed (kmean, Σ kz, Σ kz² + 1e-12; kz = k - kmean): np.unwrap
// as in unwrap_slope, the fit's two sums Σ phi and Σ kz·phi accumulated while each thread rewrites its
// run, one reduction; slope = (Σ kz·phi - mean(phi)·Σ kz) / (Σ kz² + 1e-12)  (= Σ kz·(phi - mean) / ...).
__device__ double unwrap_slope_fast(const double* ph, const int32_t* bins, int U, double kmean, double skz, double den,
                                    double* red, double* scan_tot) {
    const int per = (U + BW - 1) / BW;
    const int u0 = be_tid() * per, u1 = min(U, u0 + per);
    double local = 0.0;
    for (int u = max(u0, 1); u < u1; ++u) {
        const double dd = ph[u] - ph[u - 1];
        if (!(fabs(dd) < M_PI)) {
            double dm = np_mod(dd + M_PI, 2.0 * M_PI) - M_PI;
            if (dm == -M_PI && dd > 0.0) dm = M_PI;
            local += dm - dd;
        }
    }
    const int lane = be_tid() & 63, w = be_tid() >> 6;
    const double incl = OFS_BE_ZSCAN ? ofs::scan_add(local) : ofs::wave_scan_add(local, lane);
    if (lane == 63) scan_tot[w] = incl;
    lds_barrier();
    double run = incl - local;
    for (int k = 0; k < w; ++k) run += scan_tot[k];
    double prev_raw = u0 >= 1 && u0 < U ? ph[u0 - 1] : 0.0;
    double sv[2] = {0.0, 0.0};                               // Σ phi, Σ kz·phi
    for (int u = u0; u < u1; ++u) {
        const double raw = ph[u];
        if (u >= 1) {
            const double dd = raw - prev_raw;
            if (!(fabs(dd) < M_PI)) {
                double dm = np_mod(dd + M_PI, 2.0 * M_PI) - M_PI;
                if (dm == -M_PI && dd > 0.0) dm = M_PI;
                run += dm - dd;
            }
        }
        prev_raw = raw;
        const double phi = raw + run;
        sv[0] += phi;
        sv[1] += ((double)bins[u] - kmean) * phi;
    }
    block_sums<2>(sv, red);
    const double pmean = sv[0] / (double)U;
    return (sv[1] - pmean * skz) / den;
}

// The same fit with ONE pass over each thread's run and ONE barrier: phi(u) = raw(u) + C_t + lrun(u),
// C_t the exclusive prefix (over threads) of the thread totals of the unwrap corrections, lrun the
// thread's own running corrections, so  Σ phi = Σ_t (A_t + C_t·n_t)  and  Σ kz·phi = Σ_t (D_t + C_t·K_t)
// with A_t = Σ (raw + lrun), D_t = Σ kz·(raw + lrun), K_t = Σ kz, n_t = count over the thread's bins.
// Within a wave C_t = c_t (DPP exclusive scan) + P_w (the earlier waves' totals): each wave publishes
// (Σ A_t + c_t n_t, Σ D_t + c_t K_t, its correction total, Σ n_t, Σ K_t) and every thread combines the
// BW/64 records in wave order.  The sums associate differently from unwrap_slope_fast (slope / STO may
// differ in the last bits; the unwrap itself is the same np.unwrap per bin).  OFS_BE_UNWRAP1 = 0: the
// two-barrier form (A/B).
#ifndef OFS_BE_UNWRAP1
#define OFS_BE_UNWRAP1 1
#endif
// OFS_BE_WTOT: the records' bin counts and Σ kz are frame-invariant, so each wave's totals are scanned
// once per workgroup (be_wave_totals: the same scans of the same values, the same bits) and held as
// wave-uniform scalars; per frame only the three frame-dependent totals are scanned and published
#ifndef OFS_BE_WTOT
#define OFS_BE_WTOT 1
#endif
struct BeWaveTot { double n[BW / 64], k[BW / 64]; };
__device__ __forceinline__ double be_uniform(double v) {
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v)), hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
// each thread's run [u0, u1) as unwrap_slope_1b splits it; its count and Σ kz (the same loop order),
// scanned per wave, exchanged through LDS (slots: 2·(BW/64) doubles, callers bracket with barriers)
__device__ BeWaveTot be_wave_totals(const int32_t* bins, int U, double kmean, double* slots) {
    const int per = (U + BW - 1) / BW;
    const int u0 = be_tid() * per, u1 = min(U, u0 + per);
    double K = 0.0, cnt = 0.0;
    for (int u = u0; u < u1; ++u) {
        K += (double)bins[u] - kmean;
        cnt += 1.0;
    }
    const double sc = ofs::scan_add(cnt), sk = ofs::scan_add(K);
    const int lane = be_tid() & 63, w = be_tid() >> 6;
    if (lane == 63) {
        slots[w * 2 + 0] = sc;
        slots[w * 2 + 1] = sk;
    }
    lds_barrier();
    BeWaveTot t;
#pragma unroll
    for (int k = 0; k < BW / 64; ++k) {
        t.n[k] = be_uniform(slots[k * 2 + 0]);
        t.k[k] = be_uniform(slots[k * 2 + 1]);
    }
    lds_barrier();
    return t;
}
// OFS_BE_UNRW: the run's loop unrolled to its compile-time bound (runs are <= UPT bins) with every
// phase and bin index read up front; the same operations in the same order, bit-identical.  0: the
// runtime loop; 1: unrolled; 2 (default): unrolled for runs of 8+ bins (N 4096, 2 workgroups per CU:
// 0.8057 -> 0.8017 ms; at N 2048 / 1024 slower, 0.6407 -> 0.6478 / 0.7560 -> 0.7632, r06aq)
#ifndef OFS_BE_UNRW
#define OFS_BE_UNRW 2
#endif
template <int MAXPER>
__device__ double unwrap_slope_1b(const double* ph, const int32_t* bins, int U, double kmean, double skz, double den,
                                  double* red, double* kslot, const BeWaveTot& wt) {
    const int per = (U + BW - 1) / BW;
    const int u0 = be_tid() * per, u1 = min(U, u0 + per);
    double lrun = 0.0, A = 0.0, D = 0.0, K = 0.0, cnt = 0.0;
    double prev_raw = u0 >= 1 && u0 < U ? ph[u0 - 1] : 0.0;
    constexpr bool UNR = OFS_BE_UNRW == 1 || (OFS_BE_UNRW == 2 && MAXPER >= 8);
    if constexpr (UNR) {
    double rv[MAXPER];
    int bv[MAXPER];
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
        const int u = u0 + i;
        rv[i] = u < u1 ? ph[u] : 0.0;
        bv[i] = u < u1 ? bins[u] : 0;
    }
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
        const int u = u0 + i;
        if (u >= u1) break;
        const double raw = rv[i];
        if (u >= 1) {
            const double dd = raw - prev_raw;
            if (!(fabs(dd) < M_PI)) {
                double dm = np_mod(dd + M_PI, 2.0 * M_PI) - M_PI;
                if (dm == -M_PI && dd > 0.0) dm = M_PI;
                lrun += dm - dd;
            }
        }
        prev_raw = raw;
        const double p = raw + lrun, kz = (double)bv[i] - kmean;
        A += p;
        D += kz * p;
        K += kz;
        cnt += 1.0;
    }
    } else {
    for (int u = u0; u < u1; ++u) {
        const double raw = ph[u];
        if (u >= 1) {
            const double dd = raw - prev_raw;
            if (!(fabs(dd) < M_PI)) {
                double dm = np_mod(dd + M_PI, 2.0 * M_PI) - M_PI;
                if (dm == -M_PI && dd > 0.0) dm = M_PI;
                lrun += dm - dd;
            }
        }
        prev_raw = raw;
        const double p = raw + lrun, kz = (double)bins[u] - kmean;
        A += p;
        D += kz * p;
        K += kz;
        cnt += 1.0;
    }
    }
    const int lane = be_tid() & 63, w = be_tid() >> 6;
    const double c = ofs::scan_add(lrun) - lrun;            // exclusive wave prefix of the thread totals
    constexpr int NV = OFS_BE_WTOT ? 3 : 5;
    double v[5] = {A + c * cnt, D + c * K, lrun, cnt, K};
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = ofs::scan_add(v[i]);  // lane 63: the wave's totals
    if (lane == 63) {
#pragma unroll
        for (int i = 0; i < (OFS_BE_WTOT ? 3 : 4); ++i) red[w * 4 + i] = v[i];
        if (!OFS_BE_WTOT) kslot[w] = v[4];
    }
    lds_barrier();
    double sphi = 0.0, skzphi = 0.0, pw = 0.0;
#pragma unroll
    for (int k = 0; k < BW / 64; ++k) {
        sphi += red[k * 4 + 0] + pw * (OFS_BE_WTOT ? wt.n[k] : red[k * 4 + 3]);
        skzphi += red[k * 4 + 1] + pw * (OFS_BE_WTOT ? wt.k[k] : kslot[k]);
        pw += red[k * 4 + 2];
    }
    const double pmean = sphi / (double)U;
    return (skzphi - pmean * skz) / den;
}

#ifndef OFS_BE_MINWG
#define OFS_BE_MINWG 4             // workgroups per CU the register budget is cut for (128 VGPRs, with
                                   // the 40 KB LDS layout, OFS_BE_LDS40).  r05ab: with the lean atan2 /
                                   // sincos (be_math.h) the kernel needs 133 VGPRs, so 3 fit (0.94 ->
                                   // 0.82 ms); r05ad: 4 at 127 VGPRs (4 spilled), 0.826 -> 0.755 ms, bit-
                                   // identical.  (Round 3, with ocml's: 2 beat 3, 1.21 vs 1.29 ms.)
#endif
// LDS layout of the fast kernel's sample buffer and quarter twiddle table: both are stored with an
// XOR swizzle of the element index, so the window placement, the radix-8/8/4 passes and their
// twiddle reads are free of bank conflicts.  Identity layout: SQ_LDS_BANK_CONFLICT was 60 % of the
// kernel's LDS cycles (r05w); tools/lds_banks.py models every access (SPT 8: 5056 -> 1728 LDS
// cycles per FFT and workgroup, the conflict-free count).  Both swizzles are linear over XOR, so
// swz(p | i·h) = swz(p) ^ swz(i·h) for disjoint bit sets: a per-thread base XOR a constant.
#ifndef OFS_BE_SWZ
#define OFS_BE_SWZ 1               // 0: identity layout (A/B)
#endif
template <int SPT>
__device__ __forceinline__ constexpr int bsw(int e) {
    constexpr int LS = __builtin_ctz(SPT);
    return OFS_BE_SWZ ? e ^ ((e >> (LS + 5)) & 7) ^ (((e >> (LS + 3)) & 3) << LS) : e;
}
__device__ __forceinline__ constexpr int tsw(int j) { return OFS_BE_SWZ ? j ^ (((j >> 4) ^ (j >> 8)) & 15) : j; }

// w^j for 0 <= j < N/2 from the swizzled quarter table, given as the swizzled index of j mod N/4
// and j's quadrant bit: w^{j} = -i·w^{j-N/4}
__device__ __forceinline__ double2 twq_sw(const double2* twq, int ti, bool upper) {
    const double2 v = twq[ti];
    return upper ? make_double2(v.y, -v.x) : v;
}

// Radix-R DIT pass over groups of R·h (R = 2, 4, 8: log2 R radix-2 stages in registers): thread j
// takes the R elements p + i·h of group g = j / h, k = j mod h, and applies the stages of spans h,
// 2h, ... with the twiddles w^{(k + q·h)·N/(2·span)} - exactly the radix-2 stages' operations in
// their order (bit-identical to fft_lds), one LDS round trip and one barrier per log2 R stages.
// p and i·h have disjoint bits, as have k·str and q·h·str (k < h), so every address is a
// per-thread swizzled base XOR a compile-time constant.
template <int R, int SPT, bool WSYNC = false>
__device__ __forceinline__ void fft_pass(double2* buf, const double2* twq, int h) {
    constexpr int N = SPT * BW, Q = N / 4, LQ = __builtin_ctz(Q);
    for (int j = be_tid(); j < N / R; j += BW) {
        const int g = j / h, k = j - g * h;
        const int pb = bsw<SPT>(g * R * h + k);
        double2 v[R];
#pragma unroll
        for (int i = 0; i < R; ++i) v[i] = buf[pb ^ bsw<SPT>(i * h)];
#pragma unroll
        for (int sp = 1; sp < R; sp <<= 1) {
            const int str = N / (2 * sp * h);
            const int kk = k * str;                                   // < N / (2·sp)
            const int tb = tsw(kk & (Q - 1));
            const bool up = (kk >> LQ) & 1;
            double2 w[R / 2];
#pragma unroll
            for (int q = 0; q < sp; ++q) {
                const int qq = q * (N / (2 * sp));
                w[q] = twq_sw(twq, tb ^ tsw(qq & (Q - 1)), up != (bool)((qq >> LQ) & 1));
            }
#pragma unroll
            for (int i0 = 0; i0 < R; i0 += 2 * sp)
#pragma unroll
                for (int q = 0; q < sp; ++q) {
                    const double2 t = cmul(w[q], v[i0 + q + sp]), u = v[i0 + q];
                    v[i0 + q] = make_double2(u.x + t.x, u.y + t.y);
                    v[i0 + q + sp] = make_double2(u.x - t.x, u.y - t.y);
                }
        }
#pragma unroll
        for (int i = 0; i < R; ++i) buf[pb ^ bsw<SPT>(i * h)] = v[i];
    }
    if constexpr (WSYNC) {                 // the next pass reads only what this wave wrote (fft_rest)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        lds_barrier();
    }
}

template <int B>
__host__ __device__ constexpr int rev_bits(int v) {
    int r = 0;
    for (int i = 0; i < B; ++i) r |= ((v >> i) & 1) << (B - 1 - i);
    return r;
}
template <int V> struct Log2 { static constexpr int value = 1 + Log2<V / 2>::value; };
template <> struct Log2<1> { static constexpr int value = 0; };

// window (registers) -> rx_eff and the FFT's first log2(SPT) stages in registers -> buf.  Thread t's
// samples n = t + BW·m sit at bit-reversed positions rev(t)·SPT + rev(m): one whole group of the
// h = 1 pass, so those stages (twiddles w^{q·N/(2s)}) need no LDS round trip; the remaining 8
// stages run as radix-8, radix-8, radix-4 passes (fft_rest).
// the tone's per-BW-samples step e^{i·w0·BW/fs}: the same for both windows of a frame, so computed once
// per frame (OFS_BE_STEP1; 0: per window, A/B) - the same expression, the same bits
#ifndef OFS_BE_STEP1
#define OFS_BE_STEP1 1
#endif
__device__ __forceinline__ double2 be_tone_step(const BeArgs& a, double cfo) {
    const double w0 = 2.0 * M_PI * (-cfo);
    double ss, cc;
    ofs_bemath::sincos_lean(w0 * (double)BW / a.fs, &ss, &cc);
    return make_double2(cc, ss);
}
template <int FMT, int SPT, int NBT>
__device__ __forceinline__ void place_window_fft(const BeArgs& a, int64_t s, double cfo,
                                                 const BeWindow<FMT, SPT, NBT>& win, double2* buf,
                                                 const double2* twq, double2 step_in) {
    constexpr int N = SPT * BW, LS = Log2<SPT>::value;
    const double w0 = 2.0 * M_PI * (-cfo);
    double sn, cs;
    ofs_bemath::sincos_lean(w0 * (double)(s + (int64_t)be_tid()) / a.fs, &sn, &cs);   // core.apply_cfo's phase
    double2 tone = make_double2(cs, sn);
    const double2 step = OFS_BE_STEP1 ? step_in : be_tone_step(a, cfo);
    double2 v[SPT];
#pragma unroll
    for (int m = 0; m < SPT; ++m) {
        const int64_t i = s + be_tid() + BW * m;
        double2 acc = make_double2(0.0, 0.0);
        if (i >= 0 && i < a.T) {
#pragma unroll
            for (int r = 0; r < NBT; ++r) {
                const double2 w = cmul(widen(win.v[r][m]), tone);
                acc.x += w.x; acc.y += w.y;
            }
            acc.x /= (double)NBT; acc.y /= (double)NBT;                 // np.mean over branches
        }
        v[rev_bits<LS>(m)] = acc;
        tone = cmul(tone, step);
    }
#pragma unroll
    for (int sp = 1; sp < SPT; sp <<= 1) {                              // h = 1, k = 0
#pragma unroll
        for (int i0 = 0; i0 < SPT; i0 += 2 * sp)
#pragma unroll
            for (int q = 0; q < sp; ++q) {
                const int qq = q * (N / (2 * sp));
                const double2 w = twq_sw(twq, tsw(qq & (N / 4 - 1)), qq >= N / 4);
                const double2 t = cmul(w, v[i0 + q + sp]), u = v[i0 + q];
                v[i0 + q] = make_double2(u.x + t.x, u.y + t.y);
                v[i0 + q + sp] = make_double2(u.x - t.x, u.y - t.y);
            }
    }
    const int db = bsw<SPT>(bitrev(be_tid(), 8) * SPT);                  // bsw(i) = i for i < SPT
#pragma unroll
    for (int i = 0; i < SPT; ++i) buf[db ^ i] = v[i];
    lds_barrier();
}

// OFS_BE_WSYNC: for SPT <= 8 the first pass hands over to the second wave-locally - pass 1 thread j
// writes the 8·SPT elements of group j / SPT, pass 2 thread j reads the 64·SPT elements of group
// G = j / (8·SPT), which pass-1 threads [8·SPT·G, 8·SPT·(G + 1)) wrote: 64 (SPT 8) or 32 (SPT 4)
// threads of j's own wave (SPT 16: 128 threads, two waves - barrier)
#ifndef OFS_BE_WSYNC
#define OFS_BE_WSYNC 1
#endif
template <int SPT>
__device__ __forceinline__ void fft_rest(double2* buf, const double2* twq) {
    fft_pass<8, SPT, OFS_BE_WSYNC && SPT <= 8>(buf, twq, SPT);
    fft_pass<8, SPT>(buf, twq, 8 * SPT);
    fft_pass<4, SPT>(buf, twq, 64 * SPT);
}

#ifndef OFS_BE_PF
#define OFS_BE_PF 0                // 1: the next frame's pilot window / CP loads issued during this frame's
                                   // data phase (round 3, 0.97 vs 1.00 ms at 2 workgroups per CU; at 3:
                                   // 0.820 vs 0.823 ms with 8 VGPR spills, r05ab - off)
#endif
#ifndef OFS_BE_MINWG4
#define OFS_BE_MINWG4 5            // N = 1024 (20 KB of LDS): 5 (96 VGPRs, 4 spilled) 0.823 vs 4: 0.877 ms,
                                   // 6 (80 VGPRs): 0.827 (r05ak)
#endif
#ifndef OFS_BE_LDS40
#define OFS_BE_LDS40 1             // phases and reduction slots inside the sample buffer (0: own LDS, A/B)
#endif
#ifndef OFS_BE_MIDSLOTS
#define OFS_BE_MIDSLOTS 1          // reduction slots over the spectrum's unused Nyquist bins (below)
#endif
#ifndef OFS_BE_NOFRAMEBAR
#define OFS_BE_NOFRAMEBAR 1        // no barrier at the top of the frame loop under L40 (below)
#endif
#ifndef OFS_BE_DEARLY
#define OFS_BE_DEARLY 2            // data window loads early: 0 never, 1 always, 2 for SPT >= 16 (N 4096: 2 workgroups
#endif                             // per CU, registers to spare; r06aj 0.825 -> 0.813 ms; N 2048 / 1024 slower)
#ifndef OFS_BE_CPFIRST
#define OFS_BE_CPFIRST 0           // 1: CP loads issued before the pilot window's (A/B, r05au: 0.712 vs 0.709 ms
#endif                             // at N 2048, 0.831 vs 0.818 at 1024, 0.895 vs 0.898 at 4096 - off)
#ifndef OFS_BE_R8MAX
#define OFS_BE_R8MAX 16            // largest SPT on the register-staged radix-8 path (N = 4096: 1.049 -> 0.898 ms
                                   // with 215 VGPRs at its 2 workgroups per CU, r05as; 8: the LDS radix-4 path)
#endif
#ifndef OFS_BE_R8
#define OFS_BE_R8 1                // 0: place_window + fft_lds_q (A/B)
#endif

// (N = 4096: 80 KB of LDS, 2 workgroups per CU whatever the registers - so their budget is 256)
template <int FMT, int SPT, int NBT, int UPT>
__global__ __launch_bounds__(BW, SPT >= 16 ? 2 : (SPT <= 4 ? OFS_BE_MINWG4 : OFS_BE_MINWG)) void rx_backend_fast_kernel(BeArgs a) {
#if OFS_BE_TIMING
    long long tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    long long tprev = __builtin_amdgcn_s_memtime();
#endif
    extern __shared__ __attribute__((aligned(16))) double2 bsm[];
    constexpr int N = SPT * BW;
    double2* buf = bsm;                       // N
    double2* twq = bsm + N;                   // N / 4
#if OFS_BE_LDS40
    // LDS = the sample buffer and the twiddle table only (40 KB at N = 2048: 4 workgroups per CU):
    // the phases live in the buffer between the pilot's LS and the unwrap (the pilot spectrum is in
    // registers by then), the reduction slots at its end; barriers before each window placement
    // keep the placement's writes behind the last reads of those slots
    // OFS_BE_MIDSLOTS: the slots at the Nyquist end of the spectrum, buffer entries N/2 .. N/2 + 17 (bins
    // within [N/2, N/2 + 64) whatever the swizzle: it permutes bits below 6 only), which centered used-bin
    // sets never reach (the fast path's n_used <= N·5/8): when no used bin lies there (checked once per
    // workgroup) the EQ block sums need no barrier before their slot writes; 0: at the buffer's end (A/B)
    double* ph = reinterpret_cast<double*>(buf);                       // n_used <= N (the slots start at N)
    double* red = reinterpret_cast<double*>(buf) + (OFS_BE_MIDSLOTS ? N : 2 * N - 9 * (BW / 64));
    double* scan_tot = red + 8 * (BW / 64);
#else
    __shared__ double red[8 * (BW / 64)];
    __shared__ double scan_tot[BW / 64];
    double* ph = reinterpret_cast<double*>(twq + N / 4);   // n_used: phase / unwrap
#endif
    constexpr bool L40 = OFS_BE_LDS40;
    int rp = 0;                                               // block-sum slot set (RED2: alternating)
    auto rs = [&]() -> double* { if (OFS_BE_RED2) rp ^= 1; return red + rp * 4 * (BW / 64); };
    const int U = a.n_used, LB = 31 - __clz(N);
    constexpr bool R8 = OFS_BE_R8 && SPT <= OFS_BE_R8MAX;  // (round 3, with ocml math: 16 samples per thread spilled)
    constexpr bool PF = OFS_BE_PF && SPT <= 8 && sizeof(typename BeRaw<FMT>::T) <= 8;   // (complex128 too)
    for (int j = threadIdx.x; j < N / 4; j += BW) {
        double sn, cs;
        sincospi(-2.0 * (double)j / (double)N, &sn, &cs);
        twq[R8 ? tsw(j) : j] = make_double2(cs, sn);
    }
    int kb[UPT];                              // this thread's used bins u = tid + BW·j, as X indices
    double bsum[2] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
        const int u = threadIdx.x + BW * j;
        int k = u < U ? a.bins[u] % N : 0;
        k = k < 0 ? k + N : k;
        kb[j] = R8 ? bsw<SPT>(k) : k;                                     // buffer slot of bin k
        if (u < U) bsum[0] += (double)a.bins[u];
        if (u < U && k >= N / 2 && k < N / 2 + 64) bsum[1] = 1.0;        // a used bin under the mid slots
    }
    // the phase-slope fit's frame-invariant sums (np.mean(k), Σ kz, Σ kz² + 1e-12)
    block_sums<2>(bsum, rs());
    const double kmean = bsum[0] / (double)U;
    const bool slots_clear = L40 && OFS_BE_MIDSLOTS && bsum[1] == 0.0;   // EQ sums without the extra barrier
    double kst[2] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
        const int u = threadIdx.x + BW * j;
        if (u < U) {
            const double kz = (double)a.bins[u] - kmean;
            kst[0] += kz;
            kst[1] += kz * kz;
        }
    }
    block_sums<2>(kst, rs());
    const double skz = kst[0], kden = kst[1] + 1e-12;
    // (the slots: the reduction slot set rs() would hand out next, free until the frame loop)
    const BeWaveTot wtot = OFS_BE_WTOT ? be_wave_totals(a.bins, U, kmean, red + (rp ^ 1) * 4 * (BW / 64)) : BeWaveTot{};
    BeWindow<FMT, SPT, NBT> pwin;
    BeCp<FMT, NBT> cpx;
    // the data window's loads: issued right after the pilot window is placed (DEARLY: their HBM
    // latency hides under the pilot FFT, LS and unwrap; 32 VGPRs held meanwhile) or just before use
    constexpr bool DEARLY = (OFS_BE_DEARLY == 1 || (OFS_BE_DEARLY == 2 && SPT >= 16)) && R8;
    BeWindow<FMT, SPT, NBT> dwin;
    if (PF && blockIdx.x < a.B) {
        pwin.issue(a, blockIdx.x, a.pilot_start[blockIdx.x] + a.cp);
        cpx.issue(a, blockIdx.x, a.pilot_start[blockIdx.x]);
    }
    for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    // (L40 + OFS_BE_NOFRAMEBAR: no barrier here - the CFO block sums write the other slot set than the
    // previous frame's last sums, RED2, and the barrier before the pilot window's placement orders every
    // earlier LDS read behind it)
    if (!(L40 && OFS_BE_NOFRAMEBAR && OFS_BE_RED2)) lds_barrier();
    const int64_t ps = a.pilot_start[b], ds = a.data_start[b];
    if (!PF) {                        // (CPFIRST: the CFO would wait for the CP samples alone - vmcnt
        if (OFS_BE_CPFIRST) {         // counts in order - with the pilot window's loads still in flight)
            cpx.issue(a, b, ps);
            pwin.issue(a, b, ps + a.cp);
        } else {
            pwin.issue(a, b, ps + a.cp);
            cpx.issue(a, b, ps);
        }
    }
    double cfo;
    if (a.cfo_in) {
        cfo = a.cfo_in[b];
    } else {
        double pp[2] = {0.0, 0.0};
#pragma unroll
        for (int r = 0; r < NBT; ++r)
#pragma unroll
            for (int m = 0; m < BE_CPT; ++m) {
                const double2 u = widen(cpx.u[r][m]), v = widen(cpx.w[r][m]);
                pp[0] += u.x * v.x + u.y * v.y;
                pp[1] += u.y * v.x - u.x * v.y;
            }
        block_sums<2>(pp, rs());
        cfo = -ofs_bemath::atan2_lean(pp[1], pp[0]) * a.fs / (2.0 * M_PI * (double)N);
    }
    if (a.cfo_out && be_tid() == 0) a.cfo_out[b] = cfo;
    const double2 tstep = OFS_BE_STEP1 && R8 ? be_tone_step(a, cfo) : make_double2(0.0, 0.0);
    const double2* pil = a.pilot + b * a.pilot_stride;
    const double2* dat = a.data + b * a.data_stride;
    BE_T(0)
    // ---- pilot: FFT, used bins, LS estimate ----
    if constexpr (L40) lds_barrier();                                 // the CFO sums' slots are read
    if constexpr (R8) {
        place_window_fft<FMT, SPT, NBT>(a, ps + a.cp, cfo, pwin, buf, twq, tstep);
        if constexpr (DEARLY) dwin.issue(a, b, ds + a.cp);
        BE_T(1)
        fft_rest<SPT>(buf, twq);
    } else {
        place_window<FMT, SPT, NBT>(a, ps + a.cp, cfo, pwin, buf, LB);
        BE_T(1)
        fft_lds_q(buf, twq, N, LB);
    }
    BE_T(2)
    double2 hx[UPT];                                                  // h, later xhat
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
        const int u = be_tid() + BW * j;
        hx[j] = make_double2(0.0, 0.0);
        if (u < U) {
            const double2 p = pil[u];
            const double2 h = cdiv(buf[kb[j]], make_double2(p.x + 1e-9, p.y));   // y / (x + eps)
            hx[j] = h;
            if constexpr (!L40) ph[u] = ofs_bemath::atan2_lean(h.y, h.x);
            if (a.h_out) be_st(&a.h_out[b * U + u], h);
        }
    }
    if constexpr (L40) {                                              // ph overlays the pilot spectrum
        lds_barrier();
#pragma unroll
        for (int j = 0; j < UPT; ++j) {
            const int u = be_tid() + BW * j;
            if (u < U) ph[u] = ofs_bemath::atan2_lean(hx[j].y, hx[j].x);
        }
    }
    lds_barrier();
    BE_T(3)
    const double slope = (OFS_BE_UNWRAP1 && OFS_BE_RED2) ? unwrap_slope_1b<UPT>(ph, a.bins, U, kmean, skz, kden, rs(), scan_tot, wtot)
                                                         : unwrap_slope_fast(ph, a.bins, U, kmean, skz, kden, rs(), scan_tot);
    if (be_tid() == 0) {
        if (a.slope_out) a.slope_out[b] = slope;
        if (a.sto_out) a.sto_out[b] = -slope * (double)N / (2.0 * M_PI);
    }
    BE_T(4)
    // ---- data: FFT, equalise, complex-gain alignment, EVM ----
    {
        if constexpr (!DEARLY) dwin.issue(a, b, ds + a.cp);
        if constexpr (L40) lds_barrier();                             // the fit sums' slots are read
        if constexpr (R8) place_window_fft<FMT, SPT, NBT>(a, ds + a.cp, cfo, dwin, buf, twq, tstep);
        else place_window<FMT, SPT, NBT>(a, ds + a.cp, cfo, dwin, buf, LB);
    }
    if (PF && b + gridDim.x < a.B) {                           // the next frame's pilot window and
        const int64_t bn = b + gridDim.x;                             // CP samples land during this frame's
        pwin.issue(a, bn, a.pilot_start[bn] + a.cp);                  // data FFT, EQ and EVM
        cpx.issue(a, bn, a.pilot_start[bn]);
    }
    BE_T(5)
    if constexpr (R8) fft_rest<SPT>(buf, twq);
    else fft_lds_q(buf, twq, N, LB);
    BE_T(6)
    double gs[4] = {0.0, 0.0, 0.0, 0.0};                              // vdot(xhat, ref), |xhat|², |ref|²
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
        const int u = be_tid() + BW * j;
        if (u < U) {
            const double2 h = hx[j];
            const double2 xh = cdiv(buf[kb[j]], make_double2(h.x + 1e-9, h.y));   // equalize
            hx[j] = xh;
            const double2 r = dat[u];
            gs[0] += xh.x * r.x + xh.y * r.y;
            gs[1] += xh.x * r.y - xh.y * r.x;
            gs[2] += xh.x * xh.x + xh.y * xh.y;
            gs[3] += r.x * r.x + r.y * r.y;
        }
    }
    if (slots_clear) block_sums<4, false>(gs, rs());                  // (slots over unused bins only)
    else block_sums<4, L40>(gs, rs());                                // (L40: the slots overlay the data spectrum)
    const double rr = gs[3];
    BE_T(7)
    const double2 g = cdiv(make_double2(gs[0], gs[1]), make_double2(gs[2] + 1e-12, 0.0));
    double ee[1] = {0.0};
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
        const int u = be_tid() + BW * j;
        if (u < U) {
            const double2 xa = cmul(hx[j], g);
            if (a.xa_out) be_st(&a.xa_out[b * U + u], xa);
            const double2 r = dat[u];
            const double er = xa.x - r.x, ei = xa.y - r.y;
            ee[0] += er * er + ei * ei;
        }
    }
    block_sums<1>(ee, rs());
    if (be_tid() == 0) {
        const double evm = sqrt((ee[0] / (double)U) / (rr / (double)U));
        if (a.gain_out) a.gain_out[b] = g;
        if (a.evm_out) a.evm_out[b] = evm;
        if (a.evm_db_out) a.evm_db_out[b] = 20.0 * be_log10(evm + 1e-12);
    }
    BE_T(8)
    }
#if OFS_BE_TIMING
    if (be_tid() == 0)
        for (int i = 0; i < 9; ++i) atomicAdd(&be_prof[i], (unsigned long long)tacc[i]);
#endif
}

template <int FMT>
__global__ __launch_bounds__(BW) void rx_backend_kernel(BeArgs a) {
    extern __shared__ __attribute__((aligned(16))) double2 bsm[];
    __shared__ double red[BW / 64];
    __shared__ double scan_tot[BW / 64];
    double2* buf = bsm;                       // N
    double2* tw = bsm + a.N;                  // N / 2
    double2* hs = tw + a.N / 2;               // n_used: h, later xhat
    double* ph = reinterpret_cast<double*>(hs + a.n_used);   // n_used: phase / unwrap
    const int N = a.N, U = a.n_used, LB = 31 - __clz(N);
    for (int j = threadIdx.x; j < N / 2; j += BW) {             // once per workgroup
        double sn, cs;
        sincospi(-2.0 * (double)j / (double)N, &sn, &cs);
        tw[j] = make_double2(cs, sn);
    }
    for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {    // frames, grid-stride
    lds_barrier();
    // ---- CFO (core.py:179-196) or given ----
    const int64_t ps = a.pilot_start[b];
    double cfo;
    if (a.cfo_in) {
        cfo = a.cfo_in[b];
    } else {
        double pr = 0.0, pi = 0.0;
        for (int idx = threadIdx.x; idx < a.nb * a.cp; idx += BW) {
            const int br = idx / a.cp, n = idx - br * a.cp;
            const int64_t i0 = ps + n, i1 = ps + a.N + n;
            if (i0 >= 0 && i1 < a.T) {
                const double2 u = ld<FMT>(a.x, (b * a.nb + br) * a.T + i0);
                const double2 v = ld<FMT>(a.x, (b * a.nb + br) * a.T + i1);
                pr += u.x * v.x + u.y * v.y;
                pi += u.y * v.x - u.x * v.y;
            }
        }
        pr = block_sum(pr, red);
        pi = block_sum(pi, red);
        cfo = -atan2(pi, pr) * a.fs / (2.0 * M_PI * (double)a.N);
    }
    if (a.cfo_out && threadIdx.x == 0) a.cfo_out[b] = cfo;
    const double2* pil = a.pilot + b * a.pilot_stride;
    const double2* dat = a.data + b * a.data_stride;
    // ---- pilot: FFT, used bins, LS estimate ----
    load_window<FMT>(a, b, ps + a.cp, cfo, buf, LB);
    fft_lds(buf, tw, N, LB);
    for (int u = threadIdx.x; u < U; u += BW) {
        int k = a.bins[u] % N;
        if (k < 0) k += N;
        const double2 p = pil[u];
        const double2 h = cdiv(buf[k], make_double2(p.x + 1e-9, p.y));      // y / (x + eps)
        hs[u] = h;
        ph[u] = atan2(h.y, h.x);
        if (a.h_out) a.h_out[b * U + u] = h;
    }
    lds_barrier();
    // ---- phase slope (core.py:443-469) ----
    const double slope = unwrap_slope(ph, a.bins, U, red, scan_tot);
    if (threadIdx.x == 0) {
        if (a.slope_out) a.slope_out[b] = slope;
        if (a.sto_out) a.sto_out[b] = -slope * (double)N / (2.0 * M_PI);
    }
    // ---- data: FFT, equalise, complex-gain alignment, EVM ----
    load_window<FMT>(a, b, a.data_start[b] + a.cp, cfo, buf, LB);
    fft_lds(buf, tw, N, LB);
    double gr = 0.0, gi = 0.0, gx = 0.0, rr = 0.0;
    for (int u = threadIdx.x; u < U; u += BW) {
        int k = a.bins[u] % N;
        if (k < 0) k += N;
        const double2 h = hs[u];
        const double2 xh = cdiv(buf[k], make_double2(h.x + 1e-9, h.y));    // equalize
        hs[u] = xh;
        const double2 r = dat[u];
        gr += xh.x * r.x + xh.y * r.y;                                      // vdot(xhat, ref)
        gi += xh.x * r.y - xh.y * r.x;
        gx += xh.x * xh.x + xh.y * xh.y;                                    // vdot(xhat, xhat)
        rr += r.x * r.x + r.y * r.y;
    }
    gr = block_sum(gr, red); gi = block_sum(gi, red); gx = block_sum(gx, red); rr = block_sum(rr, red);
    const double2 g = cdiv(make_double2(gr, gi), make_double2(gx + 1e-12, 0.0));
    double ee = 0.0;
    for (int u = threadIdx.x; u < U; u += BW) {
        const double2 xa = cmul(hs[u], g);
        if (a.xa_out) a.xa_out[b * U + u] = xa;
        const double2 r = dat[u];
        const double er = xa.x - r.x, ei = xa.y - r.y;
        ee += er * er + ei * ei;
    }
    ee = block_sum(ee, red);
    if (threadIdx.x == 0) {
        const double evm = sqrt((ee / (double)U) / (rr / (double)U));
        if (a.gain_out) a.gain_out[b] = g;
        if (a.evm_out) a.evm_out[b] = evm;
        if (a.evm_db_out) a.evm_db_out[b] = 20.0 * log10(evm + 1e-12);
    }
    }
}

}  // namespace

extern "C" int32_t ofs_rx_backend(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                                  int32_t n_fft, int32_t cp_len, double fs_hz, const int64_t* pilot_start,
                                  const int64_t* data_start, const double* cfo_in, int32_t n_used,
                                  const int32_t* bins, const void* pilot_used, int64_t pilot_stride,
                                  const void* data_used, int64_t data_stride, double* cfo_out, void* h_out,
                                  void* xa_out, void* gain_out, double* evm_out, double* evm_db_out,
                                  double* slope_out, double* sto_out, void* stream) {
    if (!(in_fmt == OFS_C64 || in_fmt == OFS_C128 || in_fmt == OFS_CI16) || OFS_MISSING(x, B * T) || B < 0 || n_br < 1 ||
        T < 0 || n_fft < 2 || n_fft > BNMAX || (n_fft & (n_fft - 1)) || cp_len < 0 || n_used < 1 ||
        n_used > n_fft || OFS_MISSING(pilot_start, B) || OFS_MISSING(data_start, B) || !bins || !pilot_used || !data_used ||
        pilot_stride < 0 || data_stride < 0 || B > 0x7fffffff)
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    BeArgs a{in_fmt, x, B, T, n_br, n_fft, cp_len, n_used, fs_hz, pilot_start, data_start, cfo_in, bins,
             static_cast<const double2*>(pilot_used), pilot_stride, static_cast<const double2*>(data_used),
             data_stride, cfo_out, static_cast<double2*>(h_out), static_cast<double2*>(xa_out),
             static_cast<double2*>(gain_out), evm_out, evm_db_out, slope_out, sto_out};
    const size_t lds = (size_t)n_fft * 16 + (size_t)(n_fft / 2) * 16 + (size_t)n_used * 24;
    hipStream_t st = (hipStream_t)stream;
    auto launch = [&](auto kern) -> int32_t {
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return OFS_EHIP;
        // resident workgroups only; each walks frames with a grid stride (one twiddle table each)
        int dev = 0, cus = 256, per = 1;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, BW, lds) != hipSuccess)
            return OFS_EHIP;
        const int64_t grid = std::min<int64_t>(B, (int64_t)cus * std::max(per, 1));
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(BW), lds, st, a);
        return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
    };
    // variant BE_FAST=0: the generic kernel (A/B)
    const bool fast = !ofs::variant_off(ofs::V_BE_FAST) && (n_br == 1 || n_br == 2) && cp_len <= 2 * BW &&
                      ((n_fft == 4 * BW && n_used <= 3 * BW) || (n_fft == 8 * BW && n_used <= 5 * BW) ||
                       (n_fft == 16 * BW && n_used <= 10 * BW));
    if (fast) {
        const size_t lds_f = (size_t)n_fft * 16 + (size_t)(n_fft / 4) * 16 + (OFS_BE_LDS40 ? 0 : (size_t)n_used * 8) +
                             ofs::occ_lds();                       // variant OCC_LDS: occupancy A/B only
        auto launch_f = [&](auto kern) -> int32_t {
            if (lds_f > 64 * 1024 &&
                hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f) != hipSuccess)
                return OFS_EHIP;
            int dev = 0, cus = 256, per = 1;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, BW, lds_f) != hipSuccess)
                return OFS_EHIP;
            const int64_t grid = std::min<int64_t>(B, (int64_t)cus * std::max(per, 1));
            hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(BW), lds_f, st, a);
            return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
        };
#define BE_FAST(F)                                                                                   \
        switch (n_fft / BW * 10 + n_br) {                                                            \
            case 41: return launch_f(rx_backend_fast_kernel<F, 4, 1, 3>);                            \
            case 42: return launch_f(rx_backend_fast_kernel<F, 4, 2, 3>);                            \
            case 81: return launch_f(rx_backend_fast_kernel<F, 8, 1, 5>);                            \
            case 82: return launch_f(rx_backend_fast_kernel<F, 8, 2, 5>);                            \
            case 161: return launch_f(rx_backend_fast_kernel<F, 16, 1, 10>);                         \
            case 162: return launch_f(rx_backend_fast_kernel<F, 16, 2, 10>);                         \
        }
        switch (in_fmt) {
            case OFS_C64: BE_FAST(OFS_C64) break;
            case OFS_C128: BE_FAST(OFS_C128) break;
            default: BE_FAST(OFS_CI16) break;
        }
#undef BE_FAST
    }
    switch (in_fmt) {
        case OFS_C64: return launch(rx_backend_kernel<OFS_C64>);
        case OFS_C128: return launch(rx_backend_kernel<OFS_C128>);
        default: return launch(rx_backend_kernel<OFS_CI16>);
    }
}

// ------------------------------------------------------------------------------------------
// The back-end helpers one by one (include/ofdmsync.h): one 256-thread workgroup per row for
// the FFT and the row reductions, grid-stride elementwise kernels for the rest.  fp64 except
// quantize_adc's fp32 mode (numpy 2 keeps float32 there).
// ------------------------------------------------------------------------------------------
namespace {

// core.ofdm_fft_used (core.py:171-176): fft(x, n=N) (truncate / zero-pad), fftshift, gather
template <int FMT>
__global__ __launch_bounds__(BW) void fft_used_kernel(const void* x, int64_t B, int64_t T, int N, int U,
                                                      const int32_t* bins, double2* out) {
    extern __shared__ __attribute__((aligned(16))) double2 fsm[];
    double2* buf = fsm;
    double2* tw = fsm + N;
    const int LB = 31 - __clz(N);
    for (int j = threadIdx.x; j < N / 2; j += BW) {
        double sn, cs;
        sincospi(-2.0 * (double)j / (double)N, &sn, &cs);
        tw[j] = make_double2(cs, sn);
    }
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        lds_barrier();
        for (int n = threadIdx.x; n < N; n += BW)
            buf[bitrev(n, LB)] = n < T ? ld<FMT>(x, b * T + n) : make_double2(0.0, 0.0);
        lds_barrier();
        fft_lds(buf, tw, N, LB);
        for (int u = threadIdx.x; u < U; u += BW) {
            int k = bins[u] % N;
            if (k < 0) k += N;
            out[b * U + u] = buf[k];
        }
    }
}

__global__ void cdiv_eps_kernel(const double2* num, int64_t B, int64_t n, const double2* den, int64_t ds, double eps,
                                double2* out) {
    const int64_t total = B * n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / n, j = i - b * n;
        const double2 d = den[b * ds + j];
        out[i] = cdiv(num[i], make_double2(d.x + eps, d.y));       // num / (den + eps)
    }
}

// row reductions: remove_common_phase (OP 0), align_complex_gain (OP 1), evm_rms_db (OP 2)
template <int OP>
__global__ __launch_bounds__(BW) void row_kernel(const double2* x, int64_t B, int64_t n, const double2* ref,
                                                 int64_t rs, double eps, double2* out, double* r0, double2* g_out,
                                                 double* r1) {
    __shared__ double red[BW / 64];
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        const double2* xr = x + b * n;
        const double2* rr = ref ? ref + b * rs : nullptr;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        for (int64_t j = threadIdx.x; j < n; j += BW) {
            const double2 v = xr[j];
            if constexpr (OP == 0) {
                if (rr) {                                    // vdot(ref, x), vdot(ref, ref)
                    const double2 r = rr[j];
                    s0 += r.x * v.x + r.y * v.y; s1 += r.x * v.y - r.y * v.x; s2 += r.x * r.x + r.y * r.y;
                } else {
                    s0 += v.x; s1 += v.y;                    // mean(x)
                }
            } else if constexpr (OP == 1) {                  // vdot(x, ref), vdot(x, x)
                const double2 r = rr[j];
                s0 += v.x * r.x + v.y * r.y; s1 += v.x * r.y - v.y * r.x; s2 += v.x * v.x + v.y * v.y;
            } else {                                         // |x - ref|^2, |ref|^2
                const double2 r = rr[j];
                const double er = v.x - r.x, ei = v.y - r.y;
                s0 += er * er + ei * ei; s2 += r.x * r.x + r.y * r.y;
            }
        }
        s0 = block_sum(s0, red);
        s1 = block_sum(s1, red);
        s2 = block_sum(s2, red);
        double2 rot;
        if constexpr (OP == 0) {
            double cpe;
            if (rr) {
                const double2 q = cdiv(make_double2(s0, s1), make_double2(s2 + 1e-12, 0.0));
                cpe = atan2(q.y, q.x);
            } else {
                cpe = atan2(s1 / (double)n, s0 / (double)n);
            }
            if (threadIdx.x == 0 && r0) r0[b] = cpe;
            double sn, cs;
            sincos(cpe, &sn, &cs);
            rot = make_double2(cs, -sn);                     // exp(-i cpe)
        } else if constexpr (OP == 1) {
            rot = cdiv(make_double2(s0, s1), make_double2(s2 + eps, 0.0));
            if (threadIdx.x == 0 && g_out) g_out[b] = rot;
        } else {
            if (threadIdx.x == 0) {
                const double evm = sqrt((s0 / (double)n) / (s2 / (double)n));
                if (r0) r0[b] = evm;
                if (r1) r1[b] = 20.0 * log10(evm + 1e-12);
            }
        }
        if constexpr (OP != 2) {
            if (out)
                for (int64_t j = threadIdx.x; j < n; j += BW) out[b * n + j] = cmul(xr[j], rot);
        }
        lds_barrier();                                       // red reused by the next row
    }
}

__global__ __launch_bounds__(BW) void phase_slope_kernel(const double2* h, int64_t B, int U, const int32_t* bins,
                                                         int N, double* slope_out, double* sto_out) {
    extern __shared__ double psm[];
    __shared__ double red[BW / 64];
    __shared__ double scan_tot[BW / 64];
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        lds_barrier();
        for (int u = threadIdx.x; u < U; u += BW) {
            const double2 v = h[b * U + u];
            psm[u] = atan2(v.y, v.x);
        }
        lds_barrier();
        const double slope = unwrap_slope(psm, bins, U, red, scan_tot);
        if (threadIdx.x == 0) {
            if (slope_out) slope_out[b] = slope;
            if (sto_out) sto_out[b] = -slope * (double)N / (2.0 * M_PI);
        }
    }
}

// core.apply_cfo: phi = ((2 pi cfo) n) * (1 / fs), out = x * (cos phi + i sin phi)
template <int FMT>
__global__ void apply_cfo_kernel(const void* x, int64_t B, int nb, int64_t T, const double* cfo, double fs,
                                 double2* out) {
#pragma clang fp contract(off)
    const double rfs = 1.0 / fs;
    const int64_t total = B * nb * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = i / T, n = i - row * T, b = row / nb;
        const double w = (2.0 * M_PI) * cfo[b];
        const double ph = (w * (double)n) * rfs;
        double sn, cs;
        sincos(ph, &sn, &cs);
        const double2 v = ld<FMT>(x, i);
        out[i] = make_double2(v.x * cs - v.y * sn, v.x * sn + v.y * cs);
    }
}

// sync_aa.quantize_adc, one component: round(clip(v / fs, -1, 1 - 1/L) * L) / L * fs
template <class R>
__device__ __forceinline__ R adc_q(R v, R fs, R L) {
#pragma clang fp contract(off)
    R s = v / fs;
    const R hi = (R)1 - (R)1 / L;
    s = s < (R)-1 ? (R)-1 : s;                       // np.clip(x, -1, hi) = minimum(maximum(x, -1), hi)
    s = s > hi ? hi : s;
    return rint(s * L) / L * fs;
}

template <class IN, class R, class OUT>
__global__ void quantize_kernel(const IN* x, int64_t n, double full_scale, int bits, OUT* out) {
    const R fs = (R)full_scale, L = (R)(1ll << (bits - 1));
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const IN v = x[i];
        OUT o;
        o.x = adc_q<R>((R)v.x, fs, L);
        o.y = adc_q<R>((R)v.y, fs, L);
        out[i] = o;
    }
}

inline unsigned ew_grid(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65536)); }
inline unsigned row_grid(int64_t B) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(B, 8192)); }

}  // namespace

extern "C" {

int32_t ofs_fft_used(int32_t in_fmt, const void* x, int64_t B, int64_t T, int32_t n_fft, int32_t n_used,
                     const int32_t* bins, void* out, void* stream) {
    if (!(in_fmt == OFS_C64 || in_fmt == OFS_C128 || in_fmt == OFS_CI16) || OFS_MISSING(x, B * T) || B < 0 ||
        T < 0 || n_fft < 2 || n_fft > BNMAX || (n_fft & (n_fft - 1)) || n_used < 1 || !bins || OFS_MISSING(out, B))
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    const size_t lds = (size_t)n_fft * 16 + (size_t)(n_fft / 2) * 16;
    hipStream_t st = (hipStream_t)stream;
    auto launch = [&](auto kern) -> int32_t {
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return OFS_EHIP;
        hipLaunchKernelGGL(kern, dim3(row_grid(B)), dim3(BW), lds, st, x, B, T, (int)n_fft, (int)n_used, bins,
                           static_cast<double2*>(out));
        return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
    };
    switch (in_fmt) {
        case OFS_C64: return launch(fft_used_kernel<OFS_C64>);
        case OFS_C128: return launch(fft_used_kernel<OFS_C128>);
        default: return launch(fft_used_kernel<OFS_CI16>);
    }
}

int32_t ofs_cdiv_eps(const void* num, int64_t B, int64_t n, const void* den, int64_t den_stride, double eps,
                     void* out, void* stream) {
    if (B < 0 || n < 0 || den_stride < 0 || OFS_MISSING(num, B * n) || OFS_MISSING(den, B * n) ||
        OFS_MISSING(out, B * n))
        return OFS_EINVAL;
    if (B == 0 || n == 0) return OFS_OK;
    hipLaunchKernelGGL(cdiv_eps_kernel, dim3(ew_grid(B * n)), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const double2*>(num), B, n, static_cast<const double2*>(den), den_stride, eps,
                       static_cast<double2*>(out));
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_common_phase(const void* x, int64_t B, int64_t n, const void* ref, int64_t ref_stride, void* out,
                         double* cpe, void* stream) {
    if (B < 0 || n < 1 || ref_stride < 0 || OFS_MISSING(x, B) || OFS_MISSING(cpe, B)) return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipLaunchKernelGGL(row_kernel<0>, dim3(row_grid(B)), dim3(BW), 0, (hipStream_t)stream,
                       static_cast<const double2*>(x), B, n, static_cast<const double2*>(ref), ref_stride, 0.0,
                       static_cast<double2*>(out), cpe, (double2*)nullptr, (double*)nullptr);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_align_gain(const void* x, int64_t B, int64_t n, const void* ref, int64_t ref_stride, double eps,
                       void* out, void* gain, void* stream) {
    if (B < 0 || n < 0 || ref_stride < 0 || OFS_MISSING(x, B) || OFS_MISSING(ref, B) || OFS_MISSING(gain, B))
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipLaunchKernelGGL(row_kernel<1>, dim3(row_grid(B)), dim3(BW), 0, (hipStream_t)stream,
                       static_cast<const double2*>(x), B, n, static_cast<const double2*>(ref), ref_stride, eps,
                       static_cast<double2*>(out), (double*)nullptr, static_cast<double2*>(gain), (double*)nullptr);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_evm(const void* x, int64_t B, int64_t n, const void* ref, int64_t ref_stride, double* evm,
                double* evm_db, void* stream) {
    if (B < 0 || n < 0 || ref_stride < 0 || OFS_MISSING(x, B) || OFS_MISSING(ref, B)) return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipLaunchKernelGGL(row_kernel<2>, dim3(row_grid(B)), dim3(BW), 0, (hipStream_t)stream,
                       static_cast<const double2*>(x), B, n, static_cast<const double2*>(ref), ref_stride, 0.0,
                       (double2*)nullptr, evm, (double2*)nullptr, evm_db);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_phase_slope(const void* h, int64_t B, int32_t n_used, const int32_t* bins, int32_t n_fft,
                        double* slope, double* sto, void* stream) {
    if (B < 0 || n_used < 1 || n_used > 8192 || !bins || OFS_MISSING(h, B)) return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipLaunchKernelGGL(phase_slope_kernel, dim3(row_grid(B)), dim3(BW), (size_t)n_used * 8, (hipStream_t)stream,
                       static_cast<const double2*>(h), B, (int)n_used, bins, (int)n_fft, slope, sto);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_apply_cfo(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T, const double* cfo_hz,
                      double fs_hz, void* out, void* stream) {
    if (!(in_fmt == OFS_C64 || in_fmt == OFS_C128 || in_fmt == OFS_CI16) || B < 0 || n_br < 1 || T < 0 ||
        OFS_MISSING(x, B * T) || OFS_MISSING(cfo_hz, B) || OFS_MISSING(out, B * T))
        return OFS_EINVAL;
    const int64_t total = B * n_br * T;
    if (total == 0) return OFS_OK;
    hipStream_t st = (hipStream_t)stream;
    double2* o = static_cast<double2*>(out);
    switch (in_fmt) {
        case OFS_C64: hipLaunchKernelGGL(apply_cfo_kernel<OFS_C64>, dim3(ew_grid(total)), dim3(256), 0, st, x, B, (int)n_br, T, cfo_hz, fs_hz, o); break;
        case OFS_C128: hipLaunchKernelGGL(apply_cfo_kernel<OFS_C128>, dim3(ew_grid(total)), dim3(256), 0, st, x, B, (int)n_br, T, cfo_hz, fs_hz, o); break;
        default: hipLaunchKernelGGL(apply_cfo_kernel<OFS_CI16>, dim3(ew_grid(total)), dim3(256), 0, st, x, B, (int)n_br, T, cfo_hz, fs_hz, o); break;
    }
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_quantize_adc(int32_t in_fmt, const void* x, int64_t n, double full_scale, int32_t bits,
                         int32_t precision, void* out, void* stream) {
    if (!(in_fmt == OFS_C64 || in_fmt == OFS_C128) || n < 0 || bits < 1 || bits > 31 ||
        !(precision == OFS_FP32 || precision == OFS_FP64) || (precision == OFS_FP32 && in_fmt != OFS_C64) ||
        OFS_MISSING(x, n) || OFS_MISSING(out, n))
        return OFS_EINVAL;
    if (n == 0) return OFS_OK;
    hipStream_t st = (hipStream_t)stream;
    if (precision == OFS_FP32)
        hipLaunchKernelGGL((quantize_kernel<float2, float, float2>), dim3(ew_grid(n)), dim3(256), 0, st,
                           static_cast<const float2*>(x), n, full_scale, (int)bits, static_cast<float2*>(out));
    else if (in_fmt == OFS_C64)
        hipLaunchKernelGGL((quantize_kernel<float2, double, double2>), dim3(ew_grid(n)), dim3(256), 0, st,
                           static_cast<const float2*>(x), n, full_scale, (int)bits, static_cast<double2*>(out));
    else
        hipLaunchKernelGGL((quantize_kernel<double2, double, double2>), dim3(ew_grid(n)), dim3(256), 0, st,
                           static_cast<const double2*>(x), n, full_scale, (int)bits, static_cast<double2*>(out));
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

}  // extern "C"

#if OFS_BE_TIMING
// per-phase cycle totals of the fast back-end kernel since the last call (diagnostic builds)
extern "C" int ofs_be_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(be_prof), 9 * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[12] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(be_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
