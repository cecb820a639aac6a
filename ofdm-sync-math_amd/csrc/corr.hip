// corr.hip — the correlation-shaped metrics of the reference on gfx950:
//   park.park_streaming_metric        (park.py:64-114)      mirror product  Σ x[d-k]·x[d+k]
//   zc_v2 / zc matched filter         (zc_v2.py:244-271, zc.py:106-126)  Σ x[n-N+1+j]·conj(ref[j])
//   zc_freq.compute_frequency_metric  (zc_freq.py:62-99)    62-bin sliding DFT per offset
//   zc_v2 CFAR + gate                 (zc_v2.py:300-446)    sequential FSM, one wave per stream
//
// Park and the matched filter are O(T·N) direct sums (no prefix-sum form exists for a
// mirror product or a correlation against an arbitrary reference).  Both are fp64/fp32
// vector-FMA bound, not HBM bound: a workgroup stages its input tile (+ halo) in LDS once,
// every thread then owns OPT consecutive outputs and keeps the OPT-wide sliding window of
// the input in registers (one LDS load per step feeds OPT complex MACs).  The LDS tile is
// stored "phase-split" (element j at (j % OPT)·S + j / OPT) so that the per-step loads of
// a wave (addresses OPT·t + c) hit consecutive LDS words: conflict-free.
//
// zc_freq evaluates the 62 template bins of the N-point DFT of every window as a sliding
// DFT: lane = bin, W_k(s) = Σ_{j=s}^{s+N-1} x[j]·w_k^j is updated by (x[s+N]-x[s])·w_k^s
// per offset (w_k^{k(s+N)} = w_k^{ks}), with the twiddle w_k^s advanced by one complex
// multiply and re-anchored exactly (sincospi of an exact integer ratio) every 64 offsets.
// X_s[k] = conj(w_k^s)·W_k(s), so vdot(t, X_s) = Σ_k conj(t_k·w_k^s)·W_k(s).  The per-offset
// 62-lane sums are quad-reduced with DPP and finished through a 64-offset LDS transpose,
// so each lane ends up owning one offset and stores are coalesced.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <algorithm>
#include "ofdmsync.h"
#include "ofs_common.h"

namespace {

template <class R> struct C2;
template <> struct C2<float> { using T = float2; };
template <> struct C2<double> { using T = double2; };

template <int FMT, class R>
__device__ __forceinline__ typename C2<R>::T ld_c(const void* p, int64_t i) {
    typename C2<R>::T o;
    if constexpr (FMT == OFS_C64) {
        const float2 v = reinterpret_cast<const float2*>(p)[i];
        o.x = (R)v.x; o.y = (R)v.y;
    } else if constexpr (FMT == OFS_C128) {
        const double2 v = reinterpret_cast<const double2*>(p)[i];
        o.x = (R)v.x; o.y = (R)v.y;
    } else {
        const short2 v = reinterpret_cast<const short2*>(p)[i];
        o.x = (R)v.x; o.y = (R)v.y;
    }
    return o;
}

constexpr int CW = 256;          // threads per workgroup (Park, matched filter)
constexpr int OPT = 8;           // consecutive outputs per thread
constexpr int CD = CW * OPT;     // outputs per workgroup tile
constexpr int PADF = OPT;        // front pad of the staged tile (Park's backward window)

__host__ __device__ constexpr int64_t split_stride(int64_t len) { return (len + OPT - 1) / OPT | 1; }

// ------------------------------------------------------------------------------------------
// Park: P(d) = Σ_br Σ_{k<half} x[d-k]·x[d+k]; E(d) = Σ_br Σ_{k<half} |x[d+k]|²;
//       M = |P|²/max(E,1e-12)²;  d = half + i, i in [0, nout)   (park.py:76-113)
// Tile: global g in [g0, g0 + len), g0 = d0 - half + 1 - PADF, zero outside [0, T).
// Thread t, output q: backward b_q = x[d-k], forward f_q = x[d+k]; per step k one new
// backward value (q = 0) and one new forward value (q = OPT-1) come from LDS; the others
// rotate through a ring whose slot is (q ∓ k) mod OPT, resolved at compile time by
// unrolling k by OPT.
// ------------------------------------------------------------------------------------------
// Energy: the OPT outputs of a thread share all but the first / last few samples of their
// windows, so (SPLIT, half >= OPT) E_q = C + H_q + T_q with C = Σ_{k=OPT-1}^{half-1} |x[d0+k]|²
// (accumulated once, from output 0's forward values), H_q = Σ_{k=q}^{OPT-2} |x[d0+k]|² and
// T_q = Σ_{k=half}^{half+q-1} |x[d0+k]|² — sums of non-negative terms only, 2 instead of 2·OPT FMAs
// per step.
// (packed forms of the complex MAC measured no faster for fp32 - vector-type swizzles 3.95 ms, two
// inline-asm v_pk_fma_f32 with op_sel 2.67 ms, against 2.51 ms for the scalar FMAs: r02ab)
template <class R, class V>
__device__ __forceinline__ void park_mac(const V& b, const V& f, R& pr, R& pi) {
    pr = fma(b.x, f.x, fma(-b.y, f.y, pr));
    pi = fma(b.x, f.y, fma(b.y, f.x, pi));
}

template <int FMT, class R, bool SPLIT>
__global__ __launch_bounds__(CW) void park_kernel(const void* x, int64_t T, int nb, int half,
                                                  int64_t nout, R* __restrict__ Mo,
                                                  R* __restrict__ Po, R* __restrict__ Eo) {
    using V = typename C2<R>::T;
    extern __shared__ __align__(16) unsigned char smem_raw[];
    V* seg = reinterpret_cast<V*>(smem_raw);
    const int t = threadIdx.x;
    const int64_t b = blockIdx.y;
    const int64_t i0 = (int64_t)blockIdx.x * CD;
    const int64_t d0 = half + i0;
    const int64_t g0 = d0 - half + 1 - PADF;
    const int64_t len = CD + 2 * (int64_t)half - 2 + 2 * PADF;
    const int64_t S = split_stride(len);
    const int ksteps = (half + OPT - 1) / OPT * OPT;

    R pr[OPT], pi[OPT], en[OPT];
#pragma unroll
    for (int q = 0; q < OPT; ++q) { pr[q] = 0; pi[q] = 0; en[q] = 0; }

    for (int br = 0; br < nb; ++br) {
        const int64_t base = (b * nb + br) * T;
        __syncthreads();
        for (int64_t j = t; j < len; j += CW) {
            const int64_t g = g0 + j;
            V v; v.x = 0; v.y = 0;
            if (g >= 0 && g < T) v = ld_c<FMT, R>(x, base + g);
            seg[(j % OPT) * S + j / OPT] = v;
        }
        __syncthreads();
        // seg index of x[d0 + OPT*t + q + m] is PADF + half - 1 + OPT*t + q + m
        auto at = [&](int64_t j) -> V { return seg[(j % OPT) * S + j / OPT]; };
        const int64_t c0 = PADF + half - 1 + (int64_t)OPT * t;
        V bw[OPT], fw[OPT];
#pragma unroll
        for (int q = 0; q < OPT; ++q) { bw[q] = at(c0 + q); fw[q] = at(c0 + q); }
        R ce = 0;                                         // SPLIT: C of this branch
        for (int kk = 0; kk < ksteps; kk += OPT) {
#pragma unroll
            for (int u = 0; u < OPT; ++u) {
                const int k = kk + u;
                if (k < half) {
#pragma unroll
                    for (int q = 0; q < OPT; ++q) {
                        const V bq = bw[(q - u + OPT) % OPT];
                        const V fq = fw[(q + u) % OPT];
                        park_mac<R, V>(bq, fq, pr[q], pi[q]);
                        if (!SPLIT) en[q] = fma(fq.x, fq.x, fma(fq.y, fq.y, en[q]));
                    }
                    if (SPLIT && (kk > 0 || u >= OPT - 1)) {
                        const V f0 = fw[u % OPT];         // x[d0 + k]
                        ce = fma(f0.x, f0.x, fma(f0.y, f0.y, ce));
                    }
                }
                // next step: new backward x[d0+OPT t-(k+1)] into slot of b_{OPT-1},
                //            new forward  x[d0+OPT t+OPT-1+k+1] into slot of f_0
                bw[(OPT - 1 - u + OPT) % OPT] = at(c0 - (k + 1));
                fw[u % OPT] = at(c0 + OPT + k);
            }
        }
        if constexpr (SPLIT) {
            R hd[OPT], tl[OPT];                           // |x[d0+k]|², |x[d0+half+k]|², k < OPT-1
#pragma unroll
            for (int k = 0; k < OPT - 1; ++k) {
                const V h = at(c0 + k), w = at(c0 + half + k);
                hd[k] = fma(h.x, h.x, h.y * h.y);
                tl[k] = fma(w.x, w.x, w.y * w.y);
            }
            R hs = 0, ts = 0;
#pragma unroll
            for (int q = OPT - 1; q >= 0; --q) {          // H_q: suffix of hd from q
                en[q] += ce + hs;
                if (q > 0) hs += hd[q - 1];
            }
#pragma unroll
            for (int q = 1; q < OPT; ++q) { ts += tl[q - 1]; en[q] += ts; }   // T_q
        }
    }
#pragma unroll
    for (int q = 0; q < OPT; ++q) {
        const int64_t i = i0 + (int64_t)OPT * t + q;
        if (i < nout) {
            const int64_t o = b * nout + i;
            const R e = en[q] > (R)1e-12 ? en[q] : (R)1e-12;
            if (Mo) Mo[o] = (pr[q] * pr[q] + pi[q] * pi[q]) / (e * e);
            if (Po) { Po[2 * o] = pr[q]; Po[2 * o + 1] = pi[q]; }
            if (Eo) Eo[o] = en[q];
        }
    }
}

// ------------------------------------------------------------------------------------------
// ZC matched filter (np.convolve(x, conj(ref[::-1]), 'full'), zc_v2.py:244-254):
//   corr[n] = Σ_{j<N} xz[n-N+1+j]·conj(ref[j]),  n in [0, T+N-1)
//   energy window (np.convolve(|x|², ones(N)), zc_v2.py:266-268): same window, Σ |xz|²
// mode 0: raw per branch -> out [B*nb][nout]
// mode 1: zc_v2 detect_zc_preamble combine (zc_v2.py:493-500): Σ_br corr_br /
//         (|ref|·sqrt(max(E_br, 1e-12)))
// mode 2: zc.py:113-126 combine: Σ_br corr_br / (|ref|·sqrt(max(Σ_br E_br, 0) + 1e-12))
// mode 3: normalize_correlation(corr_in, x, ref) for one branch (zc_v2.py:257-271)
// mode 4: Σ_br corr_br, un-normalised (detect_zc_preamble with normalize=False, zc_v2.py:493-500)
// ------------------------------------------------------------------------------------------
struct ZcArgs {
    const void* x; int64_t T; int nb; int N; int64_t nout; int mode;
    const double2* ref; double ref_norm;
    const double2* corr_in; double2* out; double* mag;
};

template <int FMT>
__global__ __launch_bounds__(CW) void zc_mf_kernel(ZcArgs a) {
    using V = double2;
    extern __shared__ __align__(16) unsigned char smem_raw[];
    V* seg = reinterpret_cast<V*>(smem_raw);
    const int t = threadIdx.x;
    const int64_t by = blockIdx.y;                   // stream (modes 1-3) or stream*nb+br (mode 0)
    const int64_t n0 = (int64_t)blockIdx.x * CD;
    const int N = a.N;
    const int64_t g0 = n0 - N + 1;
    const int64_t len = CD + (int64_t)N - 1 + OPT;
    const int64_t S = split_stride(len);
    const int jsteps = (N + OPT - 1) / OPT * OPT;
    const int nbl = (a.mode == 0 || a.mode == 3) ? 1 : a.nb;
    const bool want_corr = a.mode != 3;

    double sr[OPT], si[OPT], se[OPT];
#pragma unroll
    for (int q = 0; q < OPT; ++q) { sr[q] = 0; si[q] = 0; se[q] = 0; }

    for (int br = 0; br < nbl; ++br) {
        const int64_t row = (a.mode == 0 || a.mode == 3) ? by : by * a.nb + br;
        const int64_t base = row * a.T;
        __syncthreads();
        for (int64_t j = t; j < len; j += CW) {
            const int64_t g = g0 + j;
            V v; v.x = 0; v.y = 0;
            if (g >= 0 && g < a.T) v = ld_c<FMT, double>(a.x, base + g);
            seg[(j % OPT) * S + j / OPT] = v;
        }
        __syncthreads();
        auto at = [&](int64_t j) -> V { return seg[(j % OPT) * S + j / OPT]; };
        const int64_t c0 = (int64_t)OPT * t;          // seg index of xz[n0 + OPT t - N + 1]
        double cr[OPT], ci[OPT], ce[OPT];
        V fw[OPT];
#pragma unroll
        for (int q = 0; q < OPT; ++q) { cr[q] = 0; ci[q] = 0; ce[q] = 0; fw[q] = at(c0 + q); }
        for (int jj = 0; jj < jsteps; jj += OPT) {
#pragma unroll
            for (int u = 0; u < OPT; ++u) {
                const int j = jj + u;
                if (j < N) {
                    const V r = a.ref[j];
#pragma unroll
                    for (int q = 0; q < OPT; ++q) {
                        const V f = fw[(q + u) % OPT];
                        if (want_corr) {                   // f * conj(r)
                            cr[q] = fma(f.x, r.x, fma(f.y, r.y, cr[q]));
                            ci[q] = fma(f.y, r.x, fma(-f.x, r.y, ci[q]));
                        }
                        ce[q] = fma(f.x, f.x, fma(f.y, f.y, ce[q]));
                    }
                }
                fw[u % OPT] = at(c0 + OPT + j);
            }
        }
#pragma unroll
        for (int q = 0; q < OPT; ++q) {
            if (a.mode == 1) {
                const double d = a.ref_norm * sqrt(ce[q] > 1e-12 ? ce[q] : 1e-12);
                sr[q] += cr[q] / d; si[q] += ci[q] / d;
            } else {
                sr[q] += cr[q]; si[q] += ci[q]; se[q] += ce[q];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < OPT; ++q) {
        const int64_t n = n0 + (int64_t)OPT * t + q;
        if (n >= a.nout) continue;
        const int64_t o = by * a.nout + n;
        double rr = sr[q], ri = si[q];
        if (a.mode == 2) {
            const double d = a.ref_norm * sqrt((se[q] > 0.0 ? se[q] : 0.0) + 1e-12);
            rr /= d; ri /= d;
        } else if (a.mode == 3) {
            const double d = a.ref_norm * sqrt(se[q] > 1e-12 ? se[q] : 1e-12);
            const V c = a.corr_in[o];
            rr = c.x / d; ri = c.y / d;
        }
        if (a.out) { V v; v.x = rr; v.y = ri; a.out[o] = v; }
        if (a.mag) a.mag[o] = hypot(rr, ri);
    }
}

// ------------------------------------------------------------------------------------------
// zc_freq sliding DFT.  One wave per (stream, chunk of offsets); lane = template bin.
// NB (branches, summed) is a template parameter so the per-branch window sums stay in
// registers.  fp64 throughout (the metric is a ratio of 62-bin sums).
// ------------------------------------------------------------------------------------------
// Workgroup = ZF_WAVES consecutive chunks of one stream.  When the chunk length divides N (N / chunk
// <= ZF_NBLK blocks per window), the chunks' initial windows are sums of chunk-long BLOCK DFTs
// B_k(m) = Σ_{j in block m} x[j] w^{kj}, and neighbouring chunks share all but one block: the
// workgroup computes its ZF_WAVES + N/chunk - 1 blocks once (spread over its waves) and each
// wave adds up its N/chunk of them (vs N samples per wave for a direct window).
#ifndef OFS_ZF_WAVES
#define OFS_ZF_WAVES 4
#endif
constexpr int ZF_WAVES = OFS_ZF_WAVES;
constexpr int ZF_NBLK = 8;
// offsets per transpose group: the [3][ZF_G][17] fp64 LDS transpose buffer per wave sets the
// occupancy (64 with 2-wave workgroups: 52 KiB = 6 waves per CU)
#ifndef OFS_ZF_G
#define OFS_ZF_G 16
#endif
constexpr int ZF_G = OFS_ZF_G;
constexpr int ZF_ANCHOR = 64;     // twiddle recurrence re-anchored exactly every ZF_ANCHOR offsets
struct ZfArgs {
    const void* x; int64_t B, T; int N, cp; int64_t noff, chunk, nchunks;
    int nbins; double t_energy; void* metric;
    int kb[64]; double tr[64], ti[64];
    int nb_all = 0, br0 = 0;          // zc_freq_kernel: branch rows b * nb_all + br0 + r (a branch group)
};
// zc_freq_kernel outputs: the metric in fp64 / fp32, or the partial sums (Re C, Im C, D) of a
// branch / template-bin group stored or added onto [B][noff][3] f64 (ofs_zc_freq_partial)
enum ZfOut : int { ZF_F64 = 0, ZF_F32 = 1, ZF_PART = 2, ZF_PART_ADD = 3 };

__device__ __forceinline__ double quad_sum(double v) {
    v += ofs::dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
    v += ofs::dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
    return v;
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// exp(-2*pi*i*m/N) for an exact integer m in [0, N)
__device__ __forceinline__ double2 twiddle(int64_t m, int N) {
    double s, c;
    sincospi(-2.0 * (double)m / (double)N, &s, &c);
    return make_double2(c, s);
}

// Σ_{j=s0}^{s0+len-1} x[j] w^{kj} for each branch (len a multiple of 64 or the tail): four
// independent accumulator / twiddle chains (samples j = 4m + p) so the dependent FMA and twiddle
// recurrences overlap; twiddles re-anchored exactly every 64 samples
template <int FMT, int NB>
__device__ __forceinline__ void zf_window(const ZfArgs& a, int64_t b, int64_t s0, int64_t len, int lane, int kb,
                                          const double2 wk, const double2 wk4, const double2 (&wkp)[3],
                                          double (&Wr)[NB], double (&Wi)[NB]) {
    const int N = a.N;
    double Pr[4][NB], Pi[4][NB];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int r = 0; r < NB; ++r) { Pr[p][r] = 0.0; Pi[p][r] = 0.0; }
    for (int64_t j0 = s0; j0 < s0 + len; j0 += 64) {
        const int cnt = (int)min((int64_t)64, s0 + len - j0);
        double xr[NB], xi[NB];
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            double2 v = make_double2(0.0, 0.0);
            if (lane < cnt) v = ld_c<FMT, double>(a.x, (b * a.nb_all + a.br0 + r) * a.T + j0 + lane);
            xr[r] = v.x; xi[r] = v.y;
        }
        double2 tw[4];
        tw[0] = twiddle(((int64_t)kb * j0) % N, N);                 // exact anchor per block
#pragma unroll
        for (int p = 1; p < 4; ++p)
            tw[p] = make_double2(tw[0].x * wkp[p - 1].x - tw[0].y * wkp[p - 1].y,
                                 tw[0].x * wkp[p - 1].y + tw[0].y * wkp[p - 1].x);
        if (cnt == 64) {
#pragma unroll 4
            for (int u = 0; u < 64; u += 4) {
#pragma unroll
                for (int p = 0; p < 4; ++p) {
#pragma unroll
                    for (int r = 0; r < NB; ++r) {
                        const double ur = ofs::readlane(xr[r], u + p), ui = ofs::readlane(xi[r], u + p);
                        Pr[p][r] = fma(ur, tw[p].x, fma(-ui, tw[p].y, Pr[p][r]));
                        Pi[p][r] = fma(ur, tw[p].y, fma(ui, tw[p].x, Pi[p][r]));
                    }
                    const double nr = tw[p].x * wk4.x - tw[p].y * wk4.y;
                    const double ni = tw[p].x * wk4.y + tw[p].y * wk4.x;
                    tw[p].x = nr; tw[p].y = ni;
                }
            }
        } else {
            double2 t = tw[0];
            for (int u = 0; u < cnt; ++u) {
#pragma unroll
                for (int r = 0; r < NB; ++r) {
                    const double ur = ofs::readlane(xr[r], u), ui = ofs::readlane(xi[r], u);
                    Pr[0][r] = fma(ur, t.x, fma(-ui, t.y, Pr[0][r]));
                    Pi[0][r] = fma(ur, t.y, fma(ui, t.x, Pi[0][r]));
                }
                const double nr = t.x * wk.x - t.y * wk.y;
                const double ni = t.x * wk.y + t.y * wk.x;
                t.x = nr; t.y = ni;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) {
        Wr[r] = (Pr[0][r] + Pr[1][r]) + (Pr[2][r] + Pr[3][r]);
        Wi[r] = (Pi[0][r] + Pi[1][r]) + (Pi[2][r] + Pi[3][r]);
    }
}

template <int FMT, int NB, int OUT>
__global__ __launch_bounds__(64 * ZF_WAVES) void zc_freq_kernel(ZfArgs a) {
    // LDS: the per-wave transpose buffers, aliased by the workgroup's block sums before the slide
    constexpr int RED = ZF_WAVES * 3 * ZF_G * 17;
    constexpr int BLK = (ZF_WAVES + ZF_NBLK - 1) * NB * 64 * 2;
    __shared__ double lds[RED > BLK ? RED : BLK];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t cgroups = (a.nchunks + ZF_WAVES - 1) / ZF_WAVES;
    const int64_t b = blockIdx.x / cgroups;
    const int64_t c_first = (blockIdx.x - b * cgroups) * ZF_WAVES;
    const int64_t c = c_first + wave;                           // my chunk (may be past the end)
    const int64_t o0 = c * a.chunk;
    const int64_t o1 = min(o0 + a.chunk, a.noff);
    const int N = a.N;
    const bool bin_live = lane < a.nbins;
    const int kb = bin_live ? a.kb[lane] : 0;
    const double tr = bin_live ? a.tr[lane] : 0.0, ti = bin_live ? a.ti[lane] : 0.0;
    const double emask = bin_live ? 1.0 : 0.0;
    const double2 wk = twiddle(kb, N);
    const double2 wk4 = twiddle((4 * (int64_t)kb) % N, N);
    const double2 wkp[3] = {wk, twiddle((2 * (int64_t)kb) % N, N), twiddle((3 * (int64_t)kb) % N, N)};

    double Wr[NB], Wi[NB];
    const int nblk = (a.chunk > 0 && N % a.chunk == 0) ? (int)(N / a.chunk) : 0;
    if (nblk >= 1 && nblk <= ZF_NBLK) {
        // ---- shared block sums: blocks c_first .. c_last + nblk - 1 of this stream, round-robin
        const int64_t c_last = min(c_first + ZF_WAVES, a.nchunks) - 1;
        const int nb_needed = (int)(c_last - c_first) + nblk;
        double2* blk = reinterpret_cast<double2*>(lds);           // [block][NB][64]
        for (int m = wave; m < nb_needed; m += ZF_WAVES) {
            double br_[NB], bi_[NB];
            zf_window<FMT, NB>(a, b, a.cp + (c_first + m) * a.chunk, a.chunk, lane, kb, wk, wk4, wkp, br_, bi_);
#pragma unroll
            for (int r = 0; r < NB; ++r) blk[(m * NB + r) * 64 + lane] = make_double2(br_[r], bi_[r]);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            double sr = 0.0, si = 0.0;
            if (c <= c_last)
                for (int q = 0; q < nblk; ++q) {
                    const double2 v = blk[((wave + q) * NB + r) * 64 + lane];
                    sr += v.x; si += v.y;
                }
            Wr[r] = sr; Wi[r] = si;
        }
        __syncthreads();                                          // blk is the transpose buffer below
        if (c > c_last) return;
    } else {
        if (c >= a.nchunks) return;                               // no barriers on this path
        zf_window<FMT, NB>(a, b, o0 + a.cp, N, lane, kb, wk, wk4, wkp, Wr, Wi);
    }
    double (*red)[ZF_G][17] = reinterpret_cast<double (*)[ZF_G][17]>(lds + wave * 3 * ZF_G * 17);

    // ---- slide over the chunk, ZF_G offsets per transpose group
    double2 tw = make_double2(1.0, 0.0);
    int64_t anchor = o0 - ZF_ANCHOR;
    for (int64_t og = o0; og < o1; og += ZF_G) {
        const int cnt = (int)min((int64_t)ZF_G, o1 - og);
        const int64_t sg = og + a.cp;
        double ar[NB], ai[NB], br_[NB], bi[NB];
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            const int64_t row = (b * a.nb_all + a.br0 + r) * a.T;
            double2 va = make_double2(0.0, 0.0), vb = make_double2(0.0, 0.0);
            if (lane < cnt) va = ld_c<FMT, double>(a.x, row + sg + lane);
            if (lane < cnt && sg + N + lane < a.T) vb = ld_c<FMT, double>(a.x, row + sg + N + lane);
            ar[r] = va.x; ai[r] = va.y; br_[r] = vb.x; bi[r] = vb.y;
        }
        if (og - anchor >= ZF_ANCHOR) { tw = twiddle(((int64_t)kb * sg) % N, N); anchor = og; }
        for (int u = 0; u < cnt; ++u) {
            double sr = 0.0, si = 0.0, e = 0.0;
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                sr += Wr[r]; si += Wi[r];
                e = fma(Wr[r], Wr[r], fma(Wi[r], Wi[r], e));
            }
            const double ttr = tr * tw.x - ti * tw.y;      // t_k * w^{ks}
            const double tti = tr * tw.y + ti * tw.x;
            double cr = ttr * sr + tti * si;              // conj(t w^{ks}) * Σ W
            double ci = ttr * si - tti * sr;
            e *= emask;
            cr = quad_sum(cr); ci = quad_sum(ci); e = quad_sum(e);
            if ((lane & 3) == 0) {
                red[0][u][lane >> 2] = cr;
                red[1][u][lane >> 2] = ci;
                red[2][u][lane >> 2] = e;
            }
#pragma unroll
            for (int r = 0; r < NB; ++r) {                // W(s+1) = W(s) + (x[s+N]-x[s]) w^{ks}
                const double dr = ofs::readlane(br_[r], u) - ofs::readlane(ar[r], u);
                const double di = ofs::readlane(bi[r], u) - ofs::readlane(ai[r], u);
                Wr[r] = fma(dr, tw.x, fma(-di, tw.y, Wr[r]));
                Wi[r] = fma(dr, tw.y, fma(di, tw.x, Wi[r]));
            }
            const double nr = tw.x * wk.x - tw.y * wk.y;
            const double ni = tw.x * wk.y + tw.y * wk.x;
            tw.x = nr; tw.y = ni;
        }
        wave_sync();
        if (lane < cnt) {
            double Cr = 0.0, Ci = 0.0, E = 0.0;
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                Cr += red[0][lane][g];
                Ci += red[1][lane][g];
                E += red[2][lane][g];
            }
            const int64_t o = b * a.noff + og + lane;
            if constexpr (OUT == ZF_PART || OUT == ZF_PART_ADD) {
                double* p = static_cast<double*>(a.metric) + 3 * o;
                if constexpr (OUT == ZF_PART_ADD) { Cr += p[0]; Ci += p[1]; E += p[2]; }
                p[0] = Cr; p[1] = Ci; p[2] = E;
            } else {
                const double den = a.t_energy * E;
                const double m = (Cr * Cr + Ci * Ci) / (den > 1e-12 ? den : 1e-12);
                if constexpr (OUT == ZF_F32) static_cast<float*>(a.metric)[o] = (float)m;
                else static_cast<double*>(a.metric)[o] = m;
            }
        }
        wave_sync();
    }
}

// ------------------------------------------------------------------------------------------
// zc_freq, few offsets per stream (cfg5: one window per sequence), fp32: pruned DFT by a
// 64 x R split.  N = 64 R, n = 64 a + c:  X[k] = Σ_c w_N^{kc} · Y_c[k mod R],
// Y_c[r] = Σ_a x[64a + c] w_R^{ra}.  Lane c loads column c (each load instruction reads 64
// consecutive samples: coalesced), runs an R-point radix-2 FFT in registers (twiddles are
// compile-time constants), and parks Y in LDS [r][c]; lane j then owns template bin k_j and
// sums its 64 column terms with an fp64 twiddle recurrence.  ~16 K complex MACs per window
// instead of 62·N for a direct DFT, and one read of the window: HBM-bound at cfg5's size.
// ------------------------------------------------------------------------------------------
constexpr double kPi = 3.14159265358979323846;
constexpr double c_sin(double x) {          // |x| <= pi, Taylor to 1e-17
    double t = x, s = x;
    for (int i = 1; i < 30; ++i) { t *= -x * x / ((2 * i) * (2 * i + 1)); s += t; }
    return s;
}
constexpr double c_cos(double x) {
    double t = 1, s = 1;
    for (int i = 1; i < 30; ++i) { t *= -x * x / ((2 * i - 1) * (2 * i)); s += t; }
    return s;
}
struct Tw64 {
    float c[32], s[32];
    constexpr Tw64() : c(), s() {
        for (int m = 0; m < 32; ++m) { c[m] = (float)c_cos(2 * kPi * m / 64); s[m] = (float)-c_sin(2 * kPi * m / 64); }
    }
};
constexpr int bitrev(int i, int bits) {
    int r = 0;
    for (int b = 0; b < bits; ++b) r |= ((i >> b) & 1) << (bits - 1 - b);
    return r;
}
constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v >> 1); }

// in-register forward DFT of R points (natural order in, natural order out)
template <int R>
__device__ __forceinline__ void fft_reg(float (&re)[R], float (&im)[R]) {
    constexpr Tw64 TW{};
    constexpr int LB = ilog2(R);
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int j = bitrev(i, LB);
        if (j > i) {
            const float tr = re[i], ti = im[i];
            re[i] = re[j]; im[i] = im[j]; re[j] = tr; im[j] = ti;
        }
    }
#pragma unroll
    for (int len = 2; len <= R; len <<= 1) {
#pragma unroll
        for (int i = 0; i < R; i += len) {
#pragma unroll
            for (int k = 0; k < len / 2; ++k) {
                const int m = k * (64 / len);                    // w_len^k = w_64^m
                const float wr = TW.c[m], wi = TW.s[m];
                const int p = i + k, q = i + k + len / 2;
                const float tr = re[q] * wr - im[q] * wi;
                const float ti = re[q] * wi + im[q] * wr;
                re[q] = re[p] - tr; im[q] = im[p] - ti;
                re[p] = re[p] + tr; im[p] = im[p] + ti;
            }
        }
    }
}

// Packed form of fft_reg for the cfg5 kernel: each point is one 2 x fp32 register pair, every
// butterfly is v_pk_mul + v_pk_fma (complex product, operands broadcast with op_sel) and two
// v_pk_add; w = 1 and w = -i are applied without multiplies.  Half the VALU of the scalar form.
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 cmul_pk(pf2 x, pf2 w) {           // x * w, complex
    const pf2 a = x.xx * w;                                        // (xr wr, xr wi)
    return __builtin_elementwise_fma(x.yy, pf2{-w.y, w.x}, a);    // + (-xi wi, xi wr)
}
template <int R>
__device__ __forceinline__ void fft_reg_pk(pf2 (&x)[R]) {
    constexpr Tw64 TW{};
    constexpr int LB = ilog2(R);
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int j = bitrev(i, LB);
        if (j > i) { const pf2 t = x[i]; x[i] = x[j]; x[j] = t; }
    }
#pragma unroll
    for (int len = 2; len <= R; len <<= 1) {
#pragma unroll
        for (int i = 0; i < R; i += len) {
#pragma unroll
            for (int k = 0; k < len / 2; ++k) {
                const int m = k * (64 / len);                      // w_len^k = w_64^m
                const int p = i + k, q = i + k + len / 2;
                pf2 t;
                if (m == 0) t = x[q];
                else if (m == 16) t = pf2{x[q].y, -x[q].x};        // * (-i)
                else t = cmul_pk(x[q], pf2{TW.c[m], TW.s[m]});
                x[q] = x[p] - t;
                x[p] = x[p] + t;
            }
        }
    }
}

constexpr int ZW_WAVES = 2;
template <int R>
__global__ __launch_bounds__(64 * ZW_WAVES) void zc_win_kernel(ZfArgs a, int nb) {
    __shared__ float2 Y[ZW_WAVES][R][65];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t item = (int64_t)blockIdx.x * ZW_WAVES + wave;
    if (item >= a.B * a.noff) return;                      // whole wave
    const int64_t b = item / a.noff;
    const int64_t o = item - b * a.noff;
    const int N = a.N;
    const bool live = lane < a.nbins;
    const int kb = live ? a.kb[lane] : 0;
    const int rj = kb & (R - 1);
    double s, c;
    sincospi(-2.0 * (double)kb / (double)N, &s, &c);       // w_N^{k}
    const double tr = live ? a.tr[lane] : 0.0, ti = live ? a.ti[lane] : 0.0;
    double cr = 0.0, ci = 0.0, e = 0.0;
    for (int br = 0; br < nb; ++br) {
        const float2* xs = reinterpret_cast<const float2*>(a.x) + (b * nb + br) * a.T + o + a.cp;
        float re[R], im[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float2 v = xs[64 * q + lane];
            re[q] = v.x; im[q] = v.y;
        }
        fft_reg<R>(re, im);
#pragma unroll
        for (int r = 0; r < R; ++r) Y[wave][r][lane] = make_float2(re[r], im[r]);
        wave_sync();
        double xr = 0.0, xi = 0.0, twr = 1.0, twi = 0.0;
        asm volatile("" : "+v"(c), "+v"(s));   // keep the recurrence in the loop (no 64-entry hoist)
        for (int col = 0; col < 64; ++col) {
            const float2 y = Y[wave][rj][col];
            xr += twr * y.x - twi * y.y;
            xi += twr * y.y + twi * y.x;
            const double nr = twr * c - twi * s;
            twi = twr * s + twi * c;
            twr = nr;
        }
        wave_sync();
        cr += tr * xr + ti * xi;                           // conj(t) * X
        ci += tr * xi - ti * xr;
        e += live ? xr * xr + xi * xi : 0.0;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        cr += __shfl_xor(cr, off, 64);
        ci += __shfl_xor(ci, off, 64);
        e += __shfl_xor(e, off, 64);
    }
    if (lane == 0) {
        const double den = a.t_energy * e;
        static_cast<float*>(a.metric)[item] = (float)((cr * cr + ci * ci) / (den > 1e-12 ? den : 1e-12));
    }
}

// ------------------------------------------------------------------------------------------
// zc_freq, N = 4096 (cfg5), fp32, no LDS transpose.  Same 64 x 64 split as zc_win_kernel
// (lane c owns column c, a 64-point FFT in registers gives Y_c[r]), but the column sums
// X[k] = Σ_c w_N^{kc} Y_c[k mod 64] are done ACROSS LANES: each lane scales its Y_c[r] by the
// twiddle of the bin living at residue r (table in LDS, built once per workgroup), then a
// reduce-scatter over the 64 lanes (permlane32/16 swaps, then DPP / swizzle xor steps) leaves
// lane j with X of the bin at residue j.  Needs the bins' residues mod 64 distinct (the PSS
// template's ±1..±31 are).  LDS holds only the 32 KiB table per workgroup, so occupancy is set
// by registers (the 64-sample column), and a persistent grid keeps loads of some waves in
// flight while others compute.
// ------------------------------------------------------------------------------------------
struct Zw64Args {
    const void* x; int64_t B, T; int cp; int64_t noff; double t_energy; float* metric;
    int kres[64];                 // bin k (mod N) whose residue k mod 64 is r, -1 if none
    double rtr[64], rti[64];      // template value of that bin
};
constexpr int Z64_WAVES = 4;

__device__ __forceinline__ float f_of(unsigned u) { return __uint_as_float(u); }
__device__ __forceinline__ unsigned u_of(float f) { return __float_as_uint(f); }

// v[i] += v[i + 32] of the partner half; afterwards v[i] in lane l stands for residue i + 32·l[5]
template <int M>
__device__ __forceinline__ void rs_swap_step(float (&v)[64]) {
#pragma unroll
    for (int i = 0; i < M; ++i) {
        if constexpr (M == 32) {
            const auto p = __builtin_amdgcn_permlane32_swap(u_of(v[i]), u_of(v[i + M]), false, false);
            v[i] = f_of(p[0]) + f_of(p[1]);
        } else {
            const auto p = __builtin_amdgcn_permlane16_swap(u_of(v[i]), u_of(v[i + M]), false, false);
            v[i] = f_of(p[0]) + f_of(p[1]);
        }
    }
}
// xor-partner step for M = 8, 4, 2, 1 (within 16-lane rows)
template <int M>
__device__ __forceinline__ float xor_lane(float s) {
    if constexpr (M == 8) return f_of(__builtin_amdgcn_mov_dpp(u_of(s), 0x128, 0xf, 0xf, false));  // row_ror:8
    if constexpr (M == 2) return f_of(__builtin_amdgcn_mov_dpp(u_of(s), 0x4E, 0xf, 0xf, false));   // quad_perm 2,3,0,1
    if constexpr (M == 1) return f_of(__builtin_amdgcn_mov_dpp(u_of(s), 0xB1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
    return f_of(__builtin_amdgcn_ds_swizzle(u_of(s), 0x1F | (M << 10)));                           // xor 4
}
template <int M>
__device__ __forceinline__ void rs_xor_step(float (&v)[64], int lane) {
    const bool hi = (lane & M) != 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const float send = hi ? v[i] : v[i + M];
        const float keep = hi ? v[i + M] : v[i];
        v[i] = keep + xor_lane<M>(send);
    }
}
__device__ __forceinline__ void reduce_scatter64(float (&v)[64], int lane) {
    rs_swap_step<32>(v);
    rs_swap_step<16>(v);
    rs_xor_step<8>(v, lane);
    rs_xor_step<4>(v, lane);
    rs_xor_step<2>(v, lane);
    rs_xor_step<1>(v, lane);
}

// LDS: twiddle table [64 residues][64 columns] + one 32 KiB window slot per wave
constexpr size_t Z64_LDS = (size_t)64 * 64 * sizeof(float2) * (1 + Z64_WAVES);

// One wave per SIMD (the 64-sample column is 128 VGPRs and the register FFT wants more): what
// keeps HBM busy is the wave's LDS-DMA prefetch of its NEXT window, issued as soon as the current
// window has been read out of its slot, so the load of window i+1 overlaps the FFT of window i.
// Windows that do not start on a 16-byte boundary (odd offsets) are loaded directly instead.
__global__ __launch_bounds__(64 * Z64_WAVES, 1) void zc_win64_kernel(Zw64Args a, int nb) {
    constexpr int N = 4096;
    extern __shared__ __attribute__((aligned(16))) float2 zsm[];
    float2 (*tw)[64] = reinterpret_cast<float2 (*)[64]>(zsm);   // [residue][column] = w_N^{k(r) c}
    for (int e = threadIdx.x; e < 64 * 64; e += 64 * Z64_WAVES) {
        const int r = e >> 6, c = e & 63;
        const int k = a.kres[r];
        float2 v = make_float2(0.f, 0.f);
        if (k >= 0) {
            double s, co;
            sincospi(-2.0 * (double)(((int64_t)k * c) % N) / (double)N, &s, &co);
            v = make_float2((float)co, (float)s);
        }
        tw[r][c] = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float2* slot = zsm + 64 * 64 * (1 + wave);                  // this wave's window slot
    const double tr = a.rtr[lane], ti = a.rti[lane];
    const double emask = a.kres[lane] >= 0 ? 1.0 : 0.0;
    const int64_t items = a.B * a.noff;
    const int64_t stride = (int64_t)gridDim.x * Z64_WAVES;
    // unit = (item, branch): the wave walks its units in order and prefetches the next one
    auto window = [&](int64_t it, int br) {
        const int64_t b = it / a.noff, o = it - b * a.noff;
        return reinterpret_cast<const float2*>(a.x) + (b * nb + br) * a.T + o + a.cp;
    };
    auto aligned = [](const float2* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    auto dma = [&](const float2* xs) {                          // 32 x 1 KiB, linear copy
#pragma unroll
        for (int j = 0; j < 32; ++j)
            ofs::lds_dma16(xs + 128 * j + 2 * lane, slot + 128 * j);      // stays in flight (ofs_common.h)
    };
    int64_t item = (int64_t)blockIdx.x * Z64_WAVES + wave;
    int br = 0;
    bool staged = false;                                        // current unit sits in the slot
    if (item < items) {
        const float2* xs = window(item, 0);
        staged = aligned(xs);
        if (staged) dma(xs);
    }
    double cr = 0.0, ci = 0.0, e = 0.0;
    while (item < items) {
        int64_t nitem = item;
        int nbr = br + 1;
        if (nbr == nb) { nbr = 0; nitem = item + stride; }
        pf2 xv[64];
        if (staged) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this unit's DMA has landed
#pragma unroll
            for (int q = 0; q < 64; ++q) {                      // column `lane`: x[64 q + lane]
                const float2 v = slot[64 * q + lane];
                xv[q] = pf2{v.x, v.y};
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // slot read out: free to refill
        } else {
            const float2* xs = window(item, br);
#pragma unroll
            for (int q = 0; q < 64; ++q) {
                const float2 v = xs[64 * q + lane];
                xv[q] = pf2{v.x, v.y};
            }
            // consume the loads here, before the next unit's DMA is issued: the compiler's own
            // vmcnt waits for them would otherwise count the (inline-asm) DMAs as well and drain them
#pragma unroll
            for (int q = 0; q < 64; ++q) asm volatile("" : "+v"(xv[q]));
        }
        staged = false;
        if (nitem < items) {                                    // prefetch the next unit
            const float2* xs = window(nitem, nbr);
            staged = aligned(xs);
            if (staged) dma(xs);
        }
        fft_reg_pk<64>(xv);                                     // Y_c[r], r = 0..63
        float re[64], im[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            const float2 w = tw[r][lane];
            const pf2 y = cmul_pk(xv[r], pf2{w.x, w.y});
            re[r] = y.x; im[r] = y.y;
        }
        reduce_scatter64(re, lane);
        reduce_scatter64(im, lane);
        const double xr = re[0], xi = im[0];                    // X of the bin at residue `lane`
        cr += tr * xr + ti * xi;                                // conj(t) * X
        ci += tr * xi - ti * xr;
        e += emask * (xr * xr + xi * xi);
        if (nbr == 0) {                                         // all branches of `item` summed
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                cr += __shfl_xor(cr, off, 64);
                ci += __shfl_xor(ci, off, 64);
                e += __shfl_xor(e, off, 64);
            }
            if (lane == 0) {
                const double den = a.t_energy * e;
                a.metric[item] = (float)((cr * cr + ci * ci) / (den > 1e-12 ? den : 1e-12));
            }
            cr = 0.0; ci = 0.0; e = 0.0;
        }
        item = nitem; br = nbr;
    }
}

// ------------------------------------------------------------------------------------------
// zc_v2 CFAR + gate (zc_v2.py:300-446), one wave per stream, sequential in sample order
// (the running sum is the reference's exact left-to-right float64 recursion, so given the
// same corr_mag the flags and local sums are bit-identical).  gate_only: use caller's
// above/valid arrays (detect_zc_peaks on an existing state).
// ------------------------------------------------------------------------------------------
struct ZdArgs {
    const double* mag; const uint8_t* above_in; const uint8_t* valid_in;
    int64_t n; int W; double tv, scale, minmag; int reflen, hyst;
    double* local_sum; double* corr_scaled; double* thresh_scaled;
    uint8_t* above; uint8_t* valid; uint8_t* gate_mask;
    int max_ev; int32_t* n_ev; int64_t* ev; double* ev_v;
};

__global__ __launch_bounds__(64) void zc_detect_kernel(ZdArgs a) {
#pragma clang fp contract(off)
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t n = a.n;
    const double* c = a.mag + b * n;
    const bool gate_only = a.above_in != nullptr;
    double acc = 0.0;
    bool open = false;
    int64_t gs = 0, pk = 0;
    double pv = 0.0;
    int low = 0, nev = 0;
    const int hl = a.hyst > 1 ? a.hyst - 1 : 0;
    int64_t* ev = a.ev ? a.ev + b * (int64_t)a.max_ev * 4 : nullptr;
    double* evv = a.ev_v ? a.ev_v + b * (int64_t)a.max_ev : nullptr;
    for (int64_t base = 0; base < n; base += 64) {
        const int64_t i = base + lane;
        const bool inb = i < n;
        const double ci = inb ? c[i] : 0.0;
        const double cold = (inb && i >= a.W) ? c[i - a.W] : 0.0;
        int abl = 0, vdl = 0;
        if (gate_only) {
            abl = inb ? (int)a.above_in[b * n + i] : 0;
            vdl = inb ? (int)a.valid_in[b * n + i] : 0;
        }
        const unsigned long long abm = __ballot(abl != 0), vdm = __ballot(vdl != 0);
        double my_acc = 0.0;
        int my_mask = 0, my_abv = 0;
        const int cnt = (int)min((int64_t)64, n - base);
        for (int u = 0; u < cnt; ++u) {
            const int64_t idx = base + u;
            const double cu = ofs::readlane(ci, u);
            bool vd, abv;
            if (gate_only) {
                vd = (vdm >> u) & 1ull;
                abv = (abm >> u) & 1ull;
            } else {
                if (idx >= a.W) acc = (acc + cu) - ofs::readlane(cold, u);
                else acc = acc + cu;
                vd = idx >= a.W;
                abv = vd && (cu * a.scale >= acc * a.tv) && (cu >= a.minmag);
            }
            if (lane == u) { my_acc = acc; my_abv = abv; my_mask = vd && open; }
            if (!vd) continue;
            if (!open) {
                if (abv) { open = true; gs = idx; pk = idx; pv = cu; low = 0; }
            } else {
                if (cu > pv) { pv = cu; pk = idx; }
                if (abv) {
                    low = 0;
                } else if (a.hyst == 0 || low >= hl) {
                    if (lane == 0 && ev && nev < a.max_ev) {
                        int64_t* r = ev + (int64_t)nev * 4;
                        r[0] = pk; r[1] = gs; r[2] = idx; r[3] = pk - a.reflen + 1 > 0 ? pk - a.reflen + 1 : 0;
                        if (evv) evv[nev] = pv;
                    }
                    ++nev;
                    open = false; pv = 0.0; low = 0;
                } else {
                    ++low;
                }
            }
        }
        if (inb) {
            const int64_t o = b * n + i;
            if (!gate_only) {
                if (a.local_sum) a.local_sum[o] = my_acc;
                if (a.corr_scaled) a.corr_scaled[o] = ci * a.scale;
                if (a.thresh_scaled) a.thresh_scaled[o] = my_acc * a.tv;
                if (a.above) a.above[o] = (uint8_t)my_abv;
                if (a.valid) a.valid[o] = (uint8_t)(i >= a.W);
            }
            if (a.gate_mask) a.gate_mask[o] = (uint8_t)my_mask;
        }
    }
    if (lane == 0) {
        if (open) {
            if (ev && nev < a.max_ev) {
                int64_t* r = ev + (int64_t)nev * 4;
                r[0] = pk; r[1] = gs; r[2] = n; r[3] = pk - a.reflen + 1 > 0 ? pk - a.reflen + 1 : 0;
                if (evv) evv[nev] = pv;
            }
            ++nev;
            if (a.gate_mask) a.gate_mask[b * n + gs] = 1;   // gate_mask[gate_start:n] (rest already set)
        }
        if (a.n_ev) a.n_ev[b] = nev;
    }
}

static bool fmt_ok(int f) { return f == OFS_C64 || f == OFS_C128 || f == OFS_CI16; }

template <class K>
static int set_lds(K k, size_t bytes) {
    if (bytes > 160 * 1024) return OFS_ETOOLONG;
    if (bytes > 64 * 1024 &&
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
        return OFS_EHIP;
    return OFS_OK;
}

template <int FMT, class R>
static int park_launch(const void* x, int64_t B, int nb, int64_t T, int half, int64_t nout,
                       void* M, void* P, void* E, hipStream_t st) {
    const int64_t len = CD + 2 * (int64_t)half - 2 + 2 * PADF;
    const size_t lds = (size_t)split_stride(len) * OPT * sizeof(typename C2<R>::T);
    // shared-window energy needs half >= OPT - 1 (variant PARK_DIRECT=1: per-output energy sums, A/B)
    const bool direct = ofs::variant_on(ofs::V_PARK_DIRECT);
    auto k = (half >= OPT - 1 && !direct) ? park_kernel<FMT, R, true> : park_kernel<FMT, R, false>;
    const int rc = set_lds(k, lds);
    if (rc) return rc;
    const dim3 grid((unsigned)((nout + CD - 1) / CD), (unsigned)B);
    hipLaunchKernelGGL(k, grid, dim3(CW), lds, st, x, T, nb, half, nout, (R*)M, (R*)P, (R*)E);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

template <int FMT>
static int zc_launch(const ZcArgs& a, int64_t rows, hipStream_t st) {
    const int64_t len = CD + (int64_t)a.N - 1 + OPT;
    const size_t lds = (size_t)split_stride(len) * OPT * sizeof(double2);
    auto k = zc_mf_kernel<FMT>;
    const int rc = set_lds(k, lds);
    if (rc) return rc;
    const dim3 grid((unsigned)((a.nout + CD - 1) / CD), (unsigned)rows);
    hipLaunchKernelGGL(k, grid, dim3(CW), lds, st, a);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

static int zw_launch(const ZfArgs& a, int nb, hipStream_t st) {
    const int64_t items = a.B * a.noff;
    const dim3 grid((unsigned)((items + ZW_WAVES - 1) / ZW_WAVES));
    switch (a.N / 64) {
        case 2: hipLaunchKernelGGL(zc_win_kernel<2>, grid, dim3(64 * ZW_WAVES), 0, st, a, nb); break;
        case 4: hipLaunchKernelGGL(zc_win_kernel<4>, grid, dim3(64 * ZW_WAVES), 0, st, a, nb); break;
        case 8: hipLaunchKernelGGL(zc_win_kernel<8>, grid, dim3(64 * ZW_WAVES), 0, st, a, nb); break;
        case 16: hipLaunchKernelGGL(zc_win_kernel<16>, grid, dim3(64 * ZW_WAVES), 0, st, a, nb); break;
        case 32: hipLaunchKernelGGL(zc_win_kernel<32>, grid, dim3(64 * ZW_WAVES), 0, st, a, nb); break;
        default: hipLaunchKernelGGL(zc_win_kernel<64>, grid, dim3(64 * ZW_WAVES), 0, st, a, nb); break;
    }
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

// N = 4096 lane-reduce kernel: residue table (false if two bins share a residue mod 64)
static bool zw64_args(const ZfArgs& a, Zw64Args& z) {
    z.x = a.x; z.B = a.B; z.T = a.T; z.cp = a.cp; z.noff = a.noff; z.t_energy = a.t_energy;
    z.metric = static_cast<float*>(a.metric);
    for (int r = 0; r < 64; ++r) { z.kres[r] = -1; z.rtr[r] = 0.0; z.rti[r] = 0.0; }
    for (int i = 0; i < a.nbins; ++i) {
        const int r = a.kb[i] & 63;
        if (z.kres[r] >= 0) return false;
        z.kres[r] = a.kb[i]; z.rtr[r] = a.tr[i]; z.rti[r] = a.ti[i];
    }
    return true;
}
static bool zw64_enabled() {            // variant ZW64=0 forces zc_win_kernel (A/B timing)
    return !ofs::variant_off(ofs::V_ZW64);
}
static int zw64_launch(const Zw64Args& z, int nb, hipStream_t st) {
    const int rc = set_lds(zc_win64_kernel, Z64_LDS);
    if (rc) return rc;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return OFS_EHIP;
    // persistent grid: one 160 KiB workgroup per CU (variant ZW64_GRID overrides, for tuning)
    const int64_t items = z.B * z.noff;
    int64_t grid = (items + Z64_WAVES - 1) / Z64_WAVES;
    const int64_t gv = ofs::variant_or(ofs::V_ZW64_GRID, 0);
    const int64_t cap = gv > 0 ? gv : cus;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(zc_win64_kernel, dim3((unsigned)grid), dim3(64 * Z64_WAVES), Z64_LDS, st, z, nb);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

// the window-FFT kernel serves fp32 calls with few offsets per stream (cfg5 shape)
static bool zw_ok(int in_fmt, int precision, int N, int64_t noff) {
    const int R = N / 64;
    return in_fmt == OFS_C64 && precision == OFS_FP32 && N % 64 == 0 && R >= 2 && R <= 64 &&
           (R & (R - 1)) == 0 && noff <= 64;
}

template <int FMT, int OUT>
static int zf_launch_out(const ZfArgs& a, int nb, hipStream_t st) {
    const int64_t groups = a.B * ((a.nchunks + ZF_WAVES - 1) / ZF_WAVES);     // a stream's chunk groups
    if (groups > 0x7fffffff) return OFS_EINVAL;
    const dim3 grid((unsigned)groups);
    switch (nb) {
        case 1: hipLaunchKernelGGL((zc_freq_kernel<FMT, 1, OUT>), grid, dim3(64 * ZF_WAVES), 0, st, a); break;
        case 2: hipLaunchKernelGGL((zc_freq_kernel<FMT, 2, OUT>), grid, dim3(64 * ZF_WAVES), 0, st, a); break;
        case 3: hipLaunchKernelGGL((zc_freq_kernel<FMT, 3, OUT>), grid, dim3(64 * ZF_WAVES), 0, st, a); break;
        default: hipLaunchKernelGGL((zc_freq_kernel<FMT, 4, OUT>), grid, dim3(64 * ZF_WAVES), 0, st, a); break;
    }
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}
template <int FMT>
static int zf_launch(const ZfArgs& a, int nb, int out, hipStream_t st) {
    switch (out) {
        case ZF_F32: return zf_launch_out<FMT, ZF_F32>(a, nb, st);
        case ZF_PART: return zf_launch_out<FMT, ZF_PART>(a, nb, st);
        case ZF_PART_ADD: return zf_launch_out<FMT, ZF_PART_ADD>(a, nb, st);
        default: return zf_launch_out<FMT, ZF_F64>(a, nb, st);
    }
}
// chunks of offsets for zc_freq_kernel: halve from ~N while the grid has fewer than 4096 chunks in
// all (variant ZF_ITEMS overrides the target)
static void zf_chunks(ZfArgs& a) {
    const int64_t zfv = ofs::variant_or(ofs::V_ZF_ITEMS, 4096);
    const int64_t zf_items = zfv > 0 ? zfv : 4096;
    int64_t chunk = ((std::max<int64_t>(a.N, 256) + 63) / 64) * 64;
    while (chunk > 256 && a.B * ((a.noff + chunk - 1) / chunk) < zf_items) chunk = ((chunk / 2 + 63) / 64) * 64;
    a.chunk = chunk;
    a.nchunks = (a.noff + chunk - 1) / chunk;
}
static int zf_dispatch(int in_fmt, ZfArgs& a, int nb, int out, hipStream_t st) {
    zf_chunks(a);
    switch (in_fmt) {
        case OFS_C64: return zf_launch<OFS_C64>(a, nb, out, st);
        case OFS_C128: return zf_launch<OFS_C128>(a, nb, out, st);
        default: return zf_launch<OFS_CI16>(a, nb, out, st);
    }
}

// metric = (C_re² + C_im²) / max(E_t·D, 1e-12) from accumulated partial sums
template <class OUTT>
__global__ __launch_bounds__(256) void zf_finish_kernel(const double* __restrict__ part, int64_t n, double e_t,
                                                        OUTT* __restrict__ metric) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double cr = part[3 * i], ci = part[3 * i + 1], den = e_t * part[3 * i + 2];
    metric[i] = (OUTT)((cr * cr + ci * ci) / (den > 1e-12 ? den : 1e-12));
}

}  // namespace

// zc_cfar.hip
int ofs_zc_cfar_try(const double* corr_mag, int64_t B, int64_t n, int W, double tv, double scale,
                    double minmag, int reflen, int hyst, double* local_sum, double* corr_scaled,
                    double* thresh_scaled, uint8_t* above, uint8_t* valid, uint8_t* gate_mask, int max_ev,
                    int32_t* n_ev, int64_t* ev, double* ev_v, hipStream_t st);

extern "C" {

int32_t ofs_park_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                        int32_t N, int32_t precision, void* M, void* P, void* E, void* stream) {
    if (!fmt_ok(in_fmt) || !(precision == OFS_FP32 || precision == OFS_FP64) || OFS_MISSING(x, B * T) || B < 0 ||
        n_br < 1 || T < 0 || N < 0)
        return OFS_EINVAL;
    const int half = N / 2;
    if (half == 0 || T < 2 * (int64_t)half + 1 || B == 0) return OFS_OK;   // empty (park.py:79-85)
    const int64_t nout = T - 2 * (int64_t)half;
    if (B > 65535) return OFS_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (precision == OFS_FP64) {
        switch (in_fmt) {
            case OFS_C64: return park_launch<OFS_C64, double>(x, B, n_br, T, half, nout, M, P, E, st);
            case OFS_C128: return park_launch<OFS_C128, double>(x, B, n_br, T, half, nout, M, P, E, st);
            default: return park_launch<OFS_CI16, double>(x, B, n_br, T, half, nout, M, P, E, st);
        }
    }
    switch (in_fmt) {
        case OFS_C64: return park_launch<OFS_C64, float>(x, B, n_br, T, half, nout, M, P, E, st);
        case OFS_C128: return park_launch<OFS_C128, float>(x, B, n_br, T, half, nout, M, P, E, st);
        default: return park_launch<OFS_CI16, float>(x, B, n_br, T, half, nout, M, P, E, st);
    }
}

int32_t ofs_zc_correlate(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                         const void* ref, int32_t N, double ref_energy, int32_t mode,
                         const void* corr_in, void* corr, double* corr_mag, void* stream) {
    if (!fmt_ok(in_fmt) || OFS_MISSING(x, B * T) || !ref || B < 0 || n_br < 1 || T < 1 || N < 1 || mode < 0 ||
        mode > 4 || (!corr && !corr_mag && B > 0) || (mode == 3 && (OFS_MISSING(corr_in, B) || n_br != 1)) ||
        ref_energy < 0)
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    ZcArgs a;
    a.x = x; a.T = T; a.nb = n_br; a.N = N; a.nout = T + N - 1; a.mode = mode;
    a.ref = (const double2*)ref; a.ref_norm = sqrt(ref_energy);
    a.corr_in = (const double2*)corr_in; a.out = (double2*)corr; a.mag = corr_mag;
    const int64_t rows = mode == 0 ? B * n_br : B;
    if (rows > 65535) return OFS_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    switch (in_fmt) {
        case OFS_C64: return zc_launch<OFS_C64>(a, rows, st);
        case OFS_C128: return zc_launch<OFS_C128>(a, rows, st);
        default: return zc_launch<OFS_CI16>(a, rows, st);
    }
}

// zc_slide.hip: the block-initialised sliding DFT (fp64 state; fp32 or fp64 metric out)
extern "C" int ofs_zc_slide_ok(int fmt, int n_br, int N, int nbins, int64_t noff);
extern "C" int ofs_zc_slide_launch(int fmt, int n_br, int out_f32, const void* x, int64_t B, int64_t T, int N, int cp,
                                   int nbins, const int* kb, const double* tr, const double* ti, double t_energy,
                                   void* metric, hipStream_t st);
static bool zs_enabled() {                 // variant ZS=0: the earlier one-chunk-per-wave kernel (A/B)
    return !ofs::variant_off(ofs::V_ZS);
}

// template bins into the kernel argument block (reduced mod N: fftshift(fft)[(N/2+k)%N] = fft[k mod N])
static void zf_bins(ZfArgs& a, int32_t n_bins, const int32_t* bin_indices, const double* template_bins) {
    const int N = a.N;
    for (int i = 0; i < 64; ++i) {
        if (i < n_bins) {
            a.kb[i] = (int)(((bin_indices[i] % N) + N) % N);
            a.tr[i] = template_bins[2 * i]; a.ti[i] = template_bins[2 * i + 1];
        } else {
            a.kb[i] = 0; a.tr[i] = 0.0; a.ti[i] = 0.0;
        }
    }
}

int32_t ofs_zc_freq_metric(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                           int32_t N, int32_t cp, int32_t precision, int32_t n_bins,
                           const int32_t* bin_indices, const double* template_bins,
                           double template_energy, void* metric, void* stream) {
    if (!fmt_ok(in_fmt) || OFS_MISSING(x, B * T) || OFS_MISSING(metric, B) || !bin_indices || !template_bins || B < 0 || n_br < 1 ||
        T < 0 || N < 1 || cp < 0 || n_bins < 1 || n_bins > 64 ||
        !(precision == OFS_FP32 || precision == OFS_FP64))
        return OFS_EINVAL;
    const int64_t noff = T - ((int64_t)N + cp) + 1;
    if (noff <= 0) return OFS_ESHORT;                      // zc_freq.py:76-78 raises
    if (B == 0) return OFS_OK;
    ZfArgs a;
    a.x = x; a.B = B; a.T = T; a.N = N; a.cp = cp; a.noff = noff;
    a.nbins = n_bins; a.t_energy = template_energy; a.metric = metric;
    a.nb_all = n_br; a.br0 = 0;
    zf_bins(a, n_bins, bin_indices, template_bins);
    hipStream_t st = (hipStream_t)stream;
    if (precision == OFS_FP32) {
        if (zw_ok(in_fmt, precision, N, noff)) {          // few offsets per stream: window FFTs
            Zw64Args z;
            if (N == 4096 && zw64_args(a, z) && zw64_enabled()) return zw64_launch(z, n_br, st);
            return zw_launch(a, n_br, st);
        }
        // many offsets: the fp64 sliding DFT, metric rounded to fp32 (its only fp32 step)
        const int r = ofs_zc_slide_launch(in_fmt, n_br, 1, x, B, T, N, cp, n_bins, a.kb, a.tr, a.ti,
                                          template_energy, metric, st);
        if (r != 0) return r == 1 ? OFS_OK : r;
        // shapes the block-initialised kernel does not take (3-4 branches, N not a multiple of 64,
        // blocks beyond LDS): the one-chunk-per-wave fp64 sliding DFT, metric rounded to fp32
        if (n_br > 4) return OFS_EINVAL;
        return zf_dispatch(in_fmt, a, n_br, ZF_F32, st);
    }
    if (zs_enabled()) {
        const int r = ofs_zc_slide_launch(in_fmt, n_br, 0, x, B, T, N, cp, n_bins, a.kb, a.tr, a.ti,
                                          template_energy, metric, st);
        if (r != 0) return r == 1 ? OFS_OK : r;
    }
    if (n_br > 4) return OFS_EINVAL;
    return zf_dispatch(in_fmt, a, n_br, ZF_F64, st);
}

int32_t ofs_zc_freq_partial(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T, int32_t br0,
                            int32_t n_grp, int32_t N, int32_t cp, int32_t n_bins, const int32_t* bin_indices,
                            const double* template_bins, int32_t accumulate, double* part, void* stream) {
    const int64_t noff_ = T - ((int64_t)N + cp) + 1;            // x: [B][n_br][T], part: [B][noff][3]
    if (!fmt_ok(in_fmt) || OFS_MISSING(x, B * n_br * T) || OFS_MISSING(part, B * (noff_ > 0 ? noff_ : 1)) ||
        !bin_indices || !template_bins || B < 0 ||
        n_br < 1 || br0 < 0 || n_grp < 1 || n_grp > 4 || br0 + n_grp > n_br || T < 0 || N < 1 || cp < 0 ||
        n_bins < 1 || n_bins > 64)
        return OFS_EINVAL;
    const int64_t noff = T - ((int64_t)N + cp) + 1;
    if (noff <= 0) return OFS_ESHORT;
    if (B == 0) return OFS_OK;
    ZfArgs a;
    a.x = x; a.B = B; a.T = T; a.N = N; a.cp = cp; a.noff = noff;
    a.nbins = n_bins; a.t_energy = 1.0; a.metric = part;
    a.nb_all = n_br; a.br0 = br0;
    zf_bins(a, n_bins, bin_indices, template_bins);
    return zf_dispatch(in_fmt, a, n_grp, accumulate ? ZF_PART_ADD : ZF_PART, (hipStream_t)stream);
}

int32_t ofs_zc_freq_finish(const double* part, int64_t B, int64_t noff, double template_energy, int32_t precision,
                           void* metric, void* stream) {
    if (B < 0 || noff < 0 || OFS_MISSING(part, B * noff) || OFS_MISSING(metric, B * noff) ||
        !(precision == OFS_FP32 || precision == OFS_FP64))
        return OFS_EINVAL;
    const int64_t n = B * noff;
    if (n == 0) return OFS_OK;
    const dim3 grid((unsigned)((n + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
    if (precision == OFS_FP32)
        hipLaunchKernelGGL(zf_finish_kernel<float>, grid, dim3(256), 0, st, part, n, template_energy, (float*)metric);
    else
        hipLaunchKernelGGL(zf_finish_kernel<double>, grid, dim3(256), 0, st, part, n, template_energy, (double*)metric);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_zc_freq_plan(int32_t in_fmt, int32_t precision, int64_t T, int32_t N, int32_t cp) {
    const int64_t noff = T - ((int64_t)N + cp) + 1;
    if (noff <= 0) return 0;
    if (precision == OFS_FP32) {
        if (zw_ok(in_fmt, precision, N, noff)) return (N == 4096 && zw64_enabled()) ? 3 : 2;
        return ofs_zc_slide_ok(in_fmt, 1, N, 62, noff) ? 5 : 6;
    }
    return (zs_enabled() && ofs_zc_slide_ok(in_fmt, 1, N, 62, noff)) ? 4 : 1;
}

int32_t ofs_zc_detect(const double* corr_mag, int64_t B, int64_t n, int32_t window_size,
                      int64_t thresh_value, int32_t thresh_frac_bits, double min_corr_mag,
                      int32_t reference_length, int32_t hysteresis, double* local_sum,
                      double* corr_scaled, double* thresh_scaled, uint8_t* above_threshold,
                      uint8_t* metric_valid, uint8_t* gate_mask, int32_t max_events,
                      int32_t* n_events, int64_t* ev_int, double* ev_peak, void* stream) {
    if (!corr_mag || B < 0 || n < 0 || thresh_frac_bits < 0 || thresh_frac_bits > 62 ||
        max_events < 0 || (max_events > 0 && !ev_int))
        return OFS_EINVAL;
    if (B == 0 || n == 0) return OFS_OK;
    ZdArgs a;
    a.mag = corr_mag; a.above_in = nullptr; a.valid_in = nullptr;
    a.n = n; a.W = window_size > 1 ? window_size : 1;          // RunningSum: max(1, W)
    a.tv = (double)thresh_value; a.scale = (double)(1ll << thresh_frac_bits); a.minmag = min_corr_mag;
    a.reflen = reference_length; a.hyst = hysteresis;
    a.local_sum = local_sum; a.corr_scaled = corr_scaled; a.thresh_scaled = thresh_scaled;
    a.above = above_threshold; a.valid = metric_valid; a.gate_mask = gate_mask;
    a.max_ev = max_events; a.n_ev = n_events; a.ev = ev_int; a.ev_v = ev_peak;
    // hysteresis >= 64: fused lane-per-stream recursion + closed-form gate (zc_cfar.hip)
    const int frc = ofs_zc_cfar_try(corr_mag, B, n, a.W, a.tv, a.scale, a.minmag, a.reflen, a.hyst, local_sum,
                                    corr_scaled, thresh_scaled, above_threshold, metric_valid, gate_mask,
                                    max_events, n_events, ev_int, ev_peak, (hipStream_t)stream);
    if (frc != 0) return frc > 0 ? OFS_OK : frc;
    hipLaunchKernelGGL(zc_detect_kernel, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_zc_gate(const double* corr_mag, const uint8_t* above_threshold, const uint8_t* metric_valid,
                    int64_t B, int64_t n, int32_t reference_length, int32_t hysteresis,
                    uint8_t* gate_mask, int32_t max_events, int32_t* n_events, int64_t* ev_int,
                    double* ev_peak, void* stream) {
    if (!corr_mag || !above_threshold || !metric_valid || B < 0 || n < 0 || max_events < 0 ||
        (max_events > 0 && !ev_int))
        return OFS_EINVAL;
    if (B == 0 || n == 0) return OFS_OK;
    ZdArgs a = {};
    a.mag = corr_mag; a.above_in = above_threshold; a.valid_in = metric_valid;
    a.n = n; a.W = 1; a.reflen = reference_length; a.hyst = hysteresis;
    a.gate_mask = gate_mask; a.max_ev = max_events; a.n_ev = n_events; a.ev = ev_int; a.ev_v = ev_peak;
    hipLaunchKernelGGL(zc_detect_kernel, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

}  // extern "C"
