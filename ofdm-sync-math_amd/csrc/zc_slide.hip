// zc_slide.hip — zc_freq.compute_frequency_metric (zc_freq.py:62-99) at EVERY offset of long
// streams: the 62 template bins of each window's N-point DFT by a sliding DFT in fp64.
//
// For window start s' = cp + s (offset s) and template bin k (w = exp(-2 pi i / N)):
//     X_s[k] = Σ_{n<N} x[s' + n] w^{kn}           (= fft(window)[k mod N], zc_freq.py:92-94)
//     X_{s+1}[k] = w^{-k} (X_s[k] + x[s' + N] - x[s'])                    (the sliding recursion)
//     metric(s) = |Σ_br Σ_k conj(t_k) X_s,br[k]|² / max(E_t Σ_br Σ_k |X_s,br[k]|², 1e-12)
//
// Work split (one workgroup = W waves = BPL·W consecutive chunks of C offsets of one stream):
//   phase 1  block DFTs  β_k(m) = Σ_{j<C} x[cp + mC + j] w^{kj}  of the workgroup's BPL·W + N/C - 1
//            blocks, one block per wave at a time (lane = bin, Horner in w^{4k} over four
//            interleaved chains, samples broadcast from LDS), kept in LDS;
//   phase 2  each wave slides BPL chunks at once (BPL = bins per lane, 8 by default): a row of
//            LPC = 64/BPL lanes owns one chunk, lane (r, j) owns bins j, j+LPC, ... (64 slots; slots
//            >= n_bins have w^{-k} = 0 and stay 0).  A chunk's initial window is
//            Σ_{q<N/C} w^{kqC} β_k(c + q) (no per-chunk N-sample sum), then C steps of the
//            recursion; per step the numerator / energy terms are summed in-lane over the lane's
//            BPL bins and across the row's LPC lanes by DPP (quad_perm, then row_half_mirror for
//            8 lanes or row_ror 4/8 for 16: every lane gets the row total), and lane (r, u mod LPC)
//            keeps step u's result for coalesced stores once per 16 steps.  More bins per lane =
//            fewer cross-lane steps per offset (BPL 4 -> 8: 21 -> ~15 VALU per offset).
// Every chunk starts from its own exact window (block sums), so the recursion runs at most C
// steps (error ~C·2^-53 relative).  fp64 state throughout; OUT = float rounds only the metric.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <stdint.h>
#include "ofdmsync.h"
#include "ofs_common.h"

namespace {

struct ZsArgs {
    const void* x; int64_t B, T; int N, cp; int64_t noff;
    int C, W;                      // chunk / block length (C | N), waves per workgroup
    int64_t nchunks, groups;       // chunks per stream, workgroups per stream
    int nbins; double t_energy; void* metric;
    int kb[64]; double tr[64], ti[64];
};

template <int FMT>
__device__ __forceinline__ double2 ldx(const void* p, int64_t i) {
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

// exp(-2 pi i m / N) for an exact integer m in [0, N)
__device__ __forceinline__ double2 twid(int64_t m, int N) {
    double s, c;
    sincospi(-2.0 * (double)m / (double)N, &s, &c);
    return make_double2(c, s);
}
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// a * b + c
__device__ __forceinline__ double2 cfma(double2 a, double2 b, double2 c) {
    return make_double2(fma(a.x, b.x, fma(-a.y, b.y, c.x)), fma(a.x, b.y, fma(a.y, b.x, c.y)));
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr int ZS_MAXW = 16;

// sum over the LPC lanes of a row (8 or 16), result in every lane of the row
template <int LPC>
__device__ __forceinline__ double row_sum(double v) {
    v += ofs::dpp_d<0xB1>(v);          // quad_perm [1,0,3,2]
    v += ofs::dpp_d<0x4E>(v);          // quad_perm [2,3,0,1]
    if constexpr (LPC == 8) {
        v += ofs::dpp_d<0x141>(v);     // row_half_mirror: lane i <-> 7 - i within 8 lanes
    } else {
        v += ofs::dpp_d<0x124>(v);     // row_ror:4
        v += ofs::dpp_d<0x128>(v);     // row_ror:8
    }
    return v;
}

constexpr int ZS_G = 16;               // steps per group (one d staging, one store round)
#ifndef OFS_ZS_UNROLL
#define OFS_ZS_UNROLL 2                // steps unrolled (tuning builds: -DOFS_ZS_UNROLL=1|4)
#endif

template <int FMT, int NB, int BPL, class OUT>
__global__ __launch_bounds__(64 * ZS_MAXW) void zc_slide_kernel(ZsArgs a) {
    constexpr int LPC = 64 / BPL;                                      // lanes per chunk row
    extern __shared__ __attribute__((aligned(16))) double2 zsm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int W = a.W, C = a.C, N = a.N, NQ = N / C;
    const int STG = C > ZS_G * BPL ? C : ZS_G * BPL;                  // per-wave staging per branch
    const int64_t b = blockIdx.x / a.groups, g = blockIdx.x - b * a.groups;
    const int64_t c0 = g * BPL * (int64_t)W;
    const int64_t c1 = min(c0 + BPL * (int64_t)W, a.nchunks);
    const int nblk = (int)(c1 - c0) + NQ - 1;
    double2* beta = zsm;                                               // [nblk][NB][64]
    double2* stg = zsm + (size_t)(BPL * W + NQ - 1) * NB * 64 + (size_t)w * NB * STG;   // per wave [NB][STG]

    // ---- phase 1: block DFTs (lane = bin slot) ----
    {
        const int kb = lane < a.nbins ? a.kb[lane] : 0;
        const double2 z = twid(kb, N), z2 = twid((2 * (int64_t)kb) % N, N), z3 = twid((3 * (int64_t)kb) % N, N);
        const double2 z4 = twid((4 * (int64_t)kb) % N, N);
        for (int m = w; m < nblk; m += W) {
            const int64_t s0 = a.cp + (c0 + m) * (int64_t)C;
#pragma unroll
            for (int r = 0; r < NB; ++r)
                for (int j = lane; j < C; j += 64) {
                    const int64_t i = s0 + j;
                    stg[r * STG + j] = i < a.T ? ldx<FMT>(a.x, (b * NB + r) * a.T + i) : make_double2(0.0, 0.0);
                }
            wave_sync();
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                double2 acc[4] = {make_double2(0.0, 0.0), make_double2(0.0, 0.0), make_double2(0.0, 0.0),
                                  make_double2(0.0, 0.0)};
                const double2* xs = stg + r * STG;
                for (int i = C / 4 - 1; i >= 0; --i) {
#pragma unroll
                    for (int p = 0; p < 4; ++p) acc[p] = cfma(acc[p], z4, xs[4 * i + p]);
                }
                double2 v = acc[0];
                v = cfma(acc[1], z, v);
                v = cfma(acc[2], z2, v);
                v = cfma(acc[3], z3, v);
                beta[(m * NB + r) * 64 + lane] = v;
            }
            wave_sync();                                               // staging reused
        }
    }
    __syncthreads();

    // ---- phase 2: BPL chunks per wave, BPL bins per lane ----
    const int row = lane / LPC, sl = lane % LPC;
    const int64_t c = c0 + BPL * (int64_t)w + row;                     // this row's chunk
    if (c0 + BPL * (int64_t)w >= c1) return;                           // no chunk for the whole wave (no
                                                                       // barrier follows)
    const bool live = c < c1;
    const int cl = live ? (int)(c - c0) : 0;                           // local block of the window start
    double2 cq[BPL], tq[BPL], X[BPL][NB];
#pragma unroll
    for (int q = 0; q < BPL; ++q) {
        const int slot = sl + LPC * q;
        const bool valid = slot < a.nbins;
        const int k = valid ? a.kb[slot] : 0;
        const double2 wk = twid(k, N);
        cq[q] = valid ? make_double2(wk.x, -wk.y) : make_double2(0.0, 0.0);   // w^{-k}; 0 holds a slot at 0
        tq[q] = valid ? make_double2(a.tr[slot], a.ti[slot]) : make_double2(0.0, 0.0);
        const double2 step = twid(((int64_t)k * C) % N, N);            // w^{kC}
        double2 t = make_double2(1.0, 0.0);
#pragma unroll
        for (int r = 0; r < NB; ++r) X[q][r] = make_double2(0.0, 0.0);
        for (int p = 0; p < NQ; ++p) {
#pragma unroll
            for (int r = 0; r < NB; ++r) X[q][r] = cfma(t, beta[((cl + p) * NB + r) * 64 + slot], X[q][r]);
            t = cmul(t, step);
        }
#pragma unroll
        for (int r = 0; r < NB; ++r)
            if (!valid) X[q][r] = make_double2(0.0, 0.0);
    }
    double2* dbuf = stg;                                               // [NB][BPL rows][ZS_G]
    const int64_t o0 = c * (int64_t)C;
    OUT* out = static_cast<OUT*>(a.metric) + b * a.noff;
    constexpr int KEEP = ZS_G / LPC;                                   // results kept per lane per group
    for (int og = 0; og < C; og += ZS_G) {
#pragma unroll
        for (int j = 0; j < KEEP; ++j) {
            const int64_t s = o0 + og + sl + LPC * j;                  // offsets of this lane's loads
            const int64_t i0 = a.cp + s;
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                double2 d = make_double2(0.0, 0.0);
                if (live && s < a.noff && i0 + N < a.T) {
                    const int64_t base = (b * NB + r) * a.T;
                    const double2 u = ldx<FMT>(a.x, base + i0 + N), v = ldx<FMT>(a.x, base + i0);
                    d = make_double2(u.x - v.x, u.y - v.y);
                }
                dbuf[(r * BPL + row) * ZS_G + sl + LPC * j] = d;
            }
        }
        wave_sync();
        double keep_n[KEEP], keep_e[KEEP];
#pragma unroll
        for (int j = 0; j < KEEP; ++j) { keep_n[j] = 0.0; keep_e[j] = 0.0; }
#pragma unroll OFS_ZS_UNROLL
        for (int u = 0; u < ZS_G; ++u) {
            double cr = 0.0, ci = 0.0, e = 0.0;
#pragma unroll
            for (int q = 0; q < BPL; ++q) {
                double sr = X[q][0].x, si = X[q][0].y;
#pragma unroll
                for (int r = 1; r < NB; ++r) { sr += X[q][r].x; si += X[q][r].y; }
                cr = fma(tq[q].x, sr, fma(tq[q].y, si, cr));           // conj(t) · Σ_br X
                ci = fma(tq[q].x, si, fma(-tq[q].y, sr, ci));
#pragma unroll
                for (int r = 0; r < NB; ++r) e = fma(X[q][r].x, X[q][r].x, fma(X[q][r].y, X[q][r].y, e));
            }
            cr = row_sum<LPC>(cr);
            ci = row_sum<LPC>(ci);
            e = row_sum<LPC>(e);
            const double n2 = fma(cr, cr, ci * ci);
#pragma unroll
            for (int j = 0; j < KEEP; ++j)
                if (u == sl + LPC * j) { keep_n[j] = n2; keep_e[j] = e; }
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                const double2 d = dbuf[(r * BPL + row) * ZS_G + u];
#pragma unroll
                for (int q = 0; q < BPL; ++q)
                    X[q][r] = cmul(make_double2(X[q][r].x + d.x, X[q][r].y + d.y), cq[q]);
            }
        }
        wave_sync();                                                   // dbuf rewritten next group
#pragma unroll
        for (int j = 0; j < KEEP; ++j) {
            const int64_t s = o0 + og + sl + LPC * j;
            if (live && s < a.noff) {
                const double den = a.t_energy * keep_e[j];
                out[s] = (OUT)(keep_n[j] / (den > 1e-12 ? den : 1e-12));
            }
        }
    }
}

}  // namespace

namespace {
template <int FMT, int NB, class OUT>
int zs_go(ZsArgs& a, size_t lds, int bpl, hipStream_t st) {
    auto kern = (NB == 2 || bpl == 4) ? zc_slide_kernel<FMT, NB, 4, OUT> : zc_slide_kernel<FMT, NB, NB == 2 ? 4 : 8, OUT>;
    static bool attr[2] = {false, false};            // the dynamic-LDS limit, once per instantiation
    if (!attr[bpl == 8]) {
        if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return OFS_EHIP;
        attr[bpl == 8] = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)(a.B * a.groups)), dim3(64 * a.W), lds, st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}
}  // namespace

namespace {
// chunk / block length C (C | N; 256 for N >= 8192 keeps the blocks per window at <= 32), waves per
// workgroup W (<= 16; 8 for two branches) and the workgroup's LDS; false if the blocks do not fit
// bins per lane of the slide: 8 for one branch (OFS_ZS_BPL=4 for the A/B), 4 for two (8 would
// exceed the 128 VGPRs of a 16-wave workgroup and spill)
int zs_bpl(int n_br) {
    const char* s = getenv("OFS_ZS_BPL");
    return (n_br == 2 || (s && atoi(s) == 4)) ? 4 : 8;
}

bool zs_plan(int n_br, int N, int bpl, int& C, int& W, size_t& lds, int64_t noff) {
    C = (N >= 8192 && N % 256 == 0) ? 256 : (N % 128 == 0 ? 128 : 64);
    const int64_t nchunks = (noff + C - 1) / C;
    W = (int)std::min<int64_t>(n_br == 1 ? 16 : 8, (nchunks + bpl - 1) / bpl);
    const int stg = C > 16 * bpl ? C : 16 * bpl;
    auto lds_of = [&](int w) { return ((size_t)(bpl * w + N / C - 1) * 64 + (size_t)w * stg) * n_br * sizeof(double2); };
    while (W > 1 && lds_of(W) > 160 * 1024) --W;
    lds = lds_of(W);
    return lds <= 160 * 1024;
}
}  // namespace

// Shapes the sliding kernel takes: N a multiple of 64, 1 or 2 branches, <= 64 template bins, the
// blocks of a window in LDS.
extern "C" int ofs_zc_slide_ok(int fmt, int n_br, int N, int nbins, int64_t noff) {
    if (!((fmt == OFS_C64 || fmt == OFS_C128 || fmt == OFS_CI16) && (n_br == 1 || n_br == 2) && N >= 64 &&
          N % 64 == 0 && nbins >= 1 && nbins <= 64 && noff > 0))
        return 0;
    int C, W;
    size_t lds;
    return zs_plan(n_br, N, zs_bpl(n_br), C, W, lds, noff) ? 1 : 0;
}

// Launch (1), unsupported shape (0) or OFS_E*.  kb: template bins already reduced mod N (host).
extern "C" int ofs_zc_slide_launch(int fmt, int n_br, int out_f32, const void* x, int64_t B, int64_t T, int N, int cp,
                                   int nbins, const int* kb, const double* tr, const double* ti, double t_energy,
                                   void* metric, hipStream_t st) {
    const int64_t noff = T - ((int64_t)N + cp) + 1;
    if (noff <= 0) return OFS_ESHORT;
    if (!ofs_zc_slide_ok(fmt, n_br, N, nbins, noff)) return 0;
    ZsArgs a;
    a.x = x; a.B = B; a.T = T; a.N = N; a.cp = cp; a.noff = noff;
    a.nbins = nbins; a.t_energy = t_energy; a.metric = metric;
    for (int i = 0; i < 64; ++i) {
        a.kb[i] = i < nbins ? kb[i] : 0;
        a.tr[i] = i < nbins ? tr[i] : 0.0;
        a.ti[i] = i < nbins ? ti[i] : 0.0;
    }
    size_t lds;
    const int bpl = zs_bpl(n_br);
    if (!zs_plan(n_br, N, bpl, a.C, a.W, lds, noff)) return 0;
    a.nchunks = (noff + a.C - 1) / a.C;
    a.groups = (a.nchunks + (int64_t)bpl * a.W - 1) / ((int64_t)bpl * a.W);
    if (a.B * a.groups > 0x7fffffff) return 0;
    const bool f = out_f32 != 0;
#define ZS_CASE(F, NBV) \
    if (fmt == F && n_br == NBV) return f ? zs_go<F, NBV, float>(a, lds, bpl, st) : zs_go<F, NBV, double>(a, lds, bpl, st);
    ZS_CASE(OFS_C64, 1) ZS_CASE(OFS_C64, 2) ZS_CASE(OFS_C128, 1) ZS_CASE(OFS_C128, 2)
    ZS_CASE(OFS_CI16, 1) ZS_CASE(OFS_CI16, 2)
#undef ZS_CASE
    return 0;
}
