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
//            DEFER (default): no per-step DPP at all - each lane parks its in-lane partials of
//            ZS_RG = 4 steps in LDS (the block-DFT region, dead once the initial windows are
//            built), then lane (r, j < 4) sums the row's partials of step j.  fp64 has no DPP
//            arithmetic (each DPP stage is 2 v_mov_dpp + 1 add), so the row sums were 27 of the
//            136 VALU per step, plus the keep selects; deferred, they cost ~6.
// Every chunk starts from its own exact window (block sums), so the recursion runs at most C
// steps (error ~C·2^-53 relative).  fp64 state throughout; OUT = float rounds only the metric.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
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
    int npairs; int pk[32], ps[32], pn[32];   // pair kernel: bins k (0 < k < N/2) and N-k at slots ps / pn
    int gblk;                                 // pair kernel: block DFTs by Goertzel pairs (else Horner per bin)
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

// DPP move into the lanes of the banks in BANK (4-lane groups of a 16-lane row), `old` elsewhere
template <int CTRL, int BANK>
__device__ __forceinline__ double dpp_d_bank(double old, double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, 0xf, BANK, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, 0xf, BANK, false);
    return __hiloint2double(hi, lo);
}

// Sums over the LPC lanes of a row of two steps' values at once (v0: step u, v1: step u + 1): the
// first stage pairs the row's lower half with its upper half and each side keeps one step (lower:
// u, upper: u + 1) and adds the partner's value of that step, so the remaining stages reduce ONE
// value: 1 + log2(LPC/2) stages for both steps instead of 2·log2(LPC).  Result: the lower half of
// the row holds Σ v0, the upper half Σ v1.
template <int LPC>
__device__ __forceinline__ double row_sum2(double v0, double v1) {
    constexpr int SWAP = LPC == 16 ? 0x128 : 0x141;   // row_ror:8 | row_half_mirror (lane i <-> 7 - i)
    constexpr int LO = LPC == 16 ? 0x3 : 0x5;         // banks of the lower half: 0,1 | 0,2
    constexpr int HI = 0xf ^ LO;
    const double keep = dpp_d_bank<0xE4, LO>(v1, v0);  // quad_perm identity: v0 in the lower half, else v1
    const double recv = dpp_d_bank<SWAP, HI>(dpp_d_bank<SWAP, LO>(v0, v0), v1);
    double v = keep + recv;
    v += ofs::dpp_d<0xB1>(v);                         // quad_perm [1,0,3,2]
    v += ofs::dpp_d<0x4E>(v);                         // quad_perm [2,3,0,1]
    if constexpr (LPC == 16) v += ofs::dpp_d<0x141>(v);   // row_half_mirror within the 8-lane half
    return v;
}

// Sums over a 16-lane row of four steps' values (v0..v3: steps u..u+3) by two reduce-scatter stages:
// row_ror:8 (lanes 0-7 keep steps u, u+1, lanes 8-15 steps u+2, u+3), then row_half_mirror (lane i
// <-> 7 - i: banks 0/2 keep the first of their two steps, banks 1/3 the second), then two quad
// stages on ONE value: 6 stages for four steps instead of 16.  Bank q of the row (lanes 4q..4q+3)
// ends with Σ v_q.
__device__ __forceinline__ double row_sum4(double v0, double v1, double v2, double v3) {
    const double k0 = dpp_d_bank<0xE4, 0x3>(v2, v0), k1 = dpp_d_bank<0xE4, 0x3>(v3, v1);
    const double a0 = k0 + dpp_d_bank<0x128, 0xC>(dpp_d_bank<0x128, 0x3>(v0, v0), v2);
    const double a1 = k1 + dpp_d_bank<0x128, 0xC>(dpp_d_bank<0x128, 0x3>(v1, v1), v3);
    double v = dpp_d_bank<0xE4, 0x5>(a1, a0) + dpp_d_bank<0x141, 0xA>(dpp_d_bank<0x141, 0x5>(a0, a0), a1);
    v += ofs::dpp_d<0xB1>(v);                         // quad_perm [1,0,3,2]
    v += ofs::dpp_d<0x4E>(v);                         // quad_perm [2,3,0,1]
    return v;
}

constexpr int ZS_G = 16;               // steps per group (one d staging, one store round)
// per-wave staging entries per branch: one block (phase 1), two half blocks (the pair kernel's
// phase 1) or ZS_G steps of d per row (phase 2)
__host__ __device__ constexpr int zs_stg(int C, int rows) {
    return C > ZS_G * rows ? (C > 128 ? C : 128) : (ZS_G * rows > 128 ? ZS_G * rows : 128);
}
// pair kernel: per-wave staging = one branch's block staging, or phase 2's d values of every branch
__host__ __device__ constexpr int zs_pair_stgw(int C, int rows, int nb) {
    return zs_stg(C, rows) > nb * rows * ZS_G ? zs_stg(C, rows) : nb * rows * ZS_G;
}
// pair kernel LDS: one branch's blocks (the workgroup's chunks + N/C - 1) + the waves' staging
__host__ __device__ constexpr size_t zs_pair_lds(int C, int N, int rows, int W, int nb) {
    return ((size_t)(rows * W + N / C - 1) * 64 + (size_t)W * zs_pair_stgw(C, rows, nb)) * 16;
}
constexpr int ZS_RG = 4;               // DEFER: steps per LDS partial round
constexpr int ZS_PS = 3 * 64 + 2;      // DEFER: doubles per step plane [cr, ci, e][64 lanes] + 16 B, so the
                                       // four summing lanes of a row read different bank groups
#ifndef OFS_ZS_UNROLL
#define OFS_ZS_UNROLL 2                // steps unrolled (tuning builds: -DOFS_ZS_UNROLL=1|4)
#endif
#ifndef OFS_ZS_DUNROLL
#define OFS_ZS_DUNROLL 1               // DEFER: steps unrolled per partial round (1 | 2 | 4)
#endif

// Phase 1 of both kernels: block DFTs β_k(m) = Σ_{j<C} x[cp + (c0+m)C + j] w^{kj} of the workgroup's
// nblk blocks into beta[m][NB][64 slots], one block per wave at a time (lane = bin slot, Horner in
// w^{4k} over four interleaved chains, samples broadcast from the wave's LDS staging).
template <int FMT, int NB>
__device__ __forceinline__ void zs_blocks(const ZsArgs& a, double2* beta, double2* stg, int STG, int64_t row0, int64_t c0,
                                          int nblk, int lane, int w) {
    const int C = a.C, N = a.N, W = a.W;
    const int kb = lane < a.nbins ? a.kb[lane] : 0;
    const double2 z = twid(kb, N), z2 = twid((2 * (int64_t)kb) % N, N), z3 = twid((3 * (int64_t)kb) % N, N);
    const double2 z4 = twid((4 * (int64_t)kb) % N, N);
    for (int m = w; m < nblk; m += W) {
        const int64_t s0 = a.cp + (c0 + m) * (int64_t)C;
#pragma unroll
        for (int r = 0; r < NB; ++r)
            for (int j = lane; j < C; j += 64) {
                const int64_t i = s0 + j;
                stg[r * STG + j] = i < a.T ? ldx<FMT>(a.x, (row0 + r) * a.T + i) : make_double2(0.0, 0.0);
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
        wave_sync();                                                   // staging reused
    }
}

// Phase 1 of the pair kernel: the same block DFTs, two bins per lane.  Lanes 0-31 take block m, lanes
// 32-63 block m+1, lane p the pair (k, N-k): four interleaved Goertzel resonators per branch run over
// the samples j = 4i + ch (frequency φ = 4θ, coefficient 2 cos φ, M = C/4 samples each; 4 VALU per
// sample for both bins against 4 per bin in the Horner form), and with u = w^{k(C-4)}, v = w^{kC}
//     Σ_i x[4i+ch] w^{±4ki} = u^{±1}·s_{M-1} - v^{±1}·s_{M-2},   β_{±k} = Σ_ch w^{±k ch}·(that)
// (the resonator's state grows at most ~M²·|x| at φ -> 0, so the error stays ~M²·2^-53 relative).
// Samples are staged 64 per block at a time, so the staging area is the per-bin kernel's.
template <int FMT, int NB>
__device__ __forceinline__ void zs_blocks_pair(const ZsArgs& a, double2* beta, double2* stg, int STG, int64_t row0,
                                               int64_t c0, int nblk, int lane, int w) {
    const int C = a.C, N = a.N, W = a.W, M = C / 4;
    const int half = lane >> 5, p = lane & 31;
    const bool valid = p < a.npairs;
    const int k = valid ? a.pk[p] : 1, sp = valid ? a.ps[p] : 0, sn = valid ? a.pn[p] : 0;
    const double c2 = 2.0 * twid((4 * (int64_t)k) % N, N).x;           // 2 cos 4θ
    const double2 u = twid(((int64_t)k * (C - 4)) % N, N), v = twid(((int64_t)k * C) % N, N);
    const double2 w1 = twid(k, N);
    for (int m0 = 2 * w; m0 < nblk; m0 += 2 * W) {
        const int m = m0 + half;
        double2 g[4][NB], h[4][NB];                                    // s_n, s_{n-1} of chain ch
#pragma unroll
        for (int ch = 0; ch < 4; ++ch)
#pragma unroll
            for (int r = 0; r < NB; ++r) { g[ch][r] = make_double2(0.0, 0.0); h[ch][r] = make_double2(0.0, 0.0); }
        for (int hb = 0; hb < C; hb += 64) {                           // 64 samples of each block
#pragma unroll
            for (int r = 0; r < NB; ++r)
                for (int j = lane; j < 128; j += 64) {
                    const int64_t i = a.cp + (c0 + m0 + (j >> 6)) * (int64_t)C + hb + (j & 63);
                    stg[r * STG + j] = i < a.T ? ldx<FMT>(a.x, (row0 + r) * a.T + i) : make_double2(0.0, 0.0);
                }
            wave_sync();
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                const double2* xs = stg + r * STG + half * 64;
#pragma unroll 2
                for (int i = 0; i < 16; i += 2) {                      // two samples per chain: g, h swap roles
#pragma unroll
                    for (int ch = 0; ch < 4; ++ch) {
                        const double2 x0 = xs[4 * i + ch], x1 = xs[4 * i + 4 + ch];
                        h[ch][r] = make_double2(fma(c2, g[ch][r].x, x0.x - h[ch][r].x), fma(c2, g[ch][r].y, x0.y - h[ch][r].y));
                        g[ch][r] = make_double2(fma(c2, h[ch][r].x, x1.x - g[ch][r].x), fma(c2, h[ch][r].y, x1.y - g[ch][r].y));
                    }
                }
            }
            wave_sync();                                               // staging reused
        }
        if (valid && m < nblk) {
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                double2 bp = make_double2(0.0, 0.0), bn = make_double2(0.0, 0.0);
#pragma unroll
                for (int ch = 3; ch >= 0; --ch) {                      // Horner in w^{±k} over the chains
                    const double2 S = g[ch][r], S1 = h[ch][r];
                    const double2 zp = make_double2(u.x * S.x - u.y * S.y - (v.x * S1.x - v.y * S1.y),
                                                    u.x * S.y + u.y * S.x - (v.x * S1.y + v.y * S1.x));
                    const double2 zn = make_double2(u.x * S.x + u.y * S.y - (v.x * S1.x + v.y * S1.y),
                                                    u.x * S.y - u.y * S.x - (v.x * S1.y - v.y * S1.x));
                    bp = ch == 3 ? zp : cfma(bp, w1, zp);
                    bn = ch == 3 ? zn : cfma(bn, make_double2(w1.x, -w1.y), zn);
                }
                beta[(m * NB + r) * 64 + sp] = bp;
                beta[(m * NB + r) * 64 + sn] = bn;
            }
        }
    }
}

// d = x[s'+N] - x[s'] of the ZS_G steps og.. of this row's chunk into dbuf[NB][rows][ZS_G]
template <int FMT, int NB, int LPC, int ROWS>
__device__ __forceinline__ void zs_stage_d(const ZsArgs& a, double2* dbuf, int64_t b, int64_t o0, int og, bool live,
                                           int row, int sl) {
#pragma unroll
    for (int j = 0; j < ZS_G / LPC; ++j) {
        const int u = sl + LPC * j;
        const int64_t s = o0 + og + u;
        const int64_t i0 = a.cp + s;
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            double2 d = make_double2(0.0, 0.0);
            if (live && s < a.noff && i0 + a.N < a.T) {
                const int64_t base = (b * NB + r) * a.T;
                const double2 p = ldx<FMT>(a.x, base + i0 + a.N), v = ldx<FMT>(a.x, base + i0);
                d = make_double2(p.x - v.x, p.y - v.y);
            }
            dbuf[(r * ROWS + row) * ZS_G + u] = d;
        }
    }
}

template <int FMT, int NB, int BPL, class OUT, bool DEFER>
__global__ __launch_bounds__(64 * ZS_MAXW) void zc_slide_kernel(ZsArgs a) {
    constexpr int LPC = 64 / BPL;                                      // lanes per chunk row
    extern __shared__ __attribute__((aligned(16))) double2 zsm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int W = a.W, C = a.C, N = a.N, NQ = N / C;
    const int STG = zs_stg(C, BPL);                                    // per-wave staging per branch
    const int64_t b = blockIdx.x / a.groups, g = blockIdx.x - b * a.groups;
    const int64_t c0 = g * BPL * (int64_t)W;
    const int64_t c1 = min(c0 + BPL * (int64_t)W, a.nchunks);
    const int nblk = (int)(c1 - c0) + NQ - 1;
    double2* beta = zsm;                                               // [nblk][NB][64]
    double2* stg = zsm + (size_t)(BPL * W + NQ - 1) * NB * 64 + (size_t)w * NB * STG;   // per wave [NB][STG]

    // ---- phase 1: block DFTs (lane = bin slot) ----
    zs_blocks<FMT, NB>(a, beta, stg, STG, b * NB, c0, nblk, lane, w);
    __syncthreads();

    // ---- phase 2: BPL chunks per wave, BPL bins per lane ----
    const int row = lane / LPC, sl = lane % LPC;
    const int64_t c = c0 + BPL * (int64_t)w + row;                     // this row's chunk
    const bool idle = c0 + BPL * (int64_t)w >= c1;                     // no chunk for the whole wave
    if (!DEFER && idle) return;                                        // (no barrier follows)
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
        for (int p = 0; p < (idle ? 0 : NQ); ++p) {
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
    if constexpr (DEFER) {
        // the block DFTs are dead once every wave has its initial windows: their region holds
        // the per-wave partials [ZS_RG steps][cr, ci, e][64 lanes] (6.1 KiB <= 8·NB·BPL/8 KiB per wave)
        __syncthreads();
        if (idle) return;
        double* part = reinterpret_cast<double*>(zsm) + (size_t)w * (ZS_RG * ZS_PS);
        constexpr int KD = ZS_G / ZS_RG;                               // partial rounds per group
        for (int og = 0; og < C; og += ZS_G) {
            zs_stage_d<FMT, NB, LPC, BPL>(a, dbuf, b, o0, og, live, row, sl);
            wave_sync();
#pragma unroll 1
            for (int v = 0; v < KD; ++v) {
#pragma unroll OFS_ZS_DUNROLL
                for (int uu = 0; uu < ZS_RG; ++uu) {
                    const int u = v * ZS_RG + uu;
                    double cr = 0.0, ci = 0.0, e = 0.0;
#pragma unroll
                    for (int q = 0; q < BPL; ++q) {
                        double sr = X[q][0].x, si = X[q][0].y;
#pragma unroll
                        for (int r = 1; r < NB; ++r) { sr += X[q][r].x; si += X[q][r].y; }
                        cr = fma(tq[q].x, sr, fma(tq[q].y, si, cr));   // conj(t) · Σ_br X
                        ci = fma(tq[q].x, si, fma(-tq[q].y, sr, ci));
#pragma unroll
                        for (int r = 0; r < NB; ++r) e = fma(X[q][r].x, X[q][r].x, fma(X[q][r].y, X[q][r].y, e));
                    }
                    part[uu * ZS_PS + lane] = cr;
                    part[uu * ZS_PS + 64 + lane] = ci;
                    part[uu * ZS_PS + 128 + lane] = e;
#pragma unroll
                    for (int r = 0; r < NB; ++r) {
                        const double2 d = dbuf[(r * BPL + row) * ZS_G + u];
#pragma unroll
                        for (int q = 0; q < BPL; ++q)
                            X[q][r] = cmul(make_double2(X[q][r].x + d.x, X[q][r].y + d.y), cq[q]);
                    }
                }
                wave_sync();
                if (sl < ZS_RG) {                                      // lane (row, j): step v·RG + j
                    const double* p = part + sl * ZS_PS + row * LPC;
                    double sr = 0.0, si = 0.0, se = 0.0;
#pragma unroll
                    for (int l = 0; l < LPC; l += 2) {
                        const double2 pr = *reinterpret_cast<const double2*>(p + l);
                        const double2 pi = *reinterpret_cast<const double2*>(p + 64 + l);
                        const double2 pe = *reinterpret_cast<const double2*>(p + 128 + l);
                        sr += pr.x + pr.y;
                        si += pi.x + pi.y;
                        se += pe.x + pe.y;
                    }
                    const int64_t s = o0 + og + v * ZS_RG + sl;
                    if (live && s < a.noff) {
                        const double den = a.t_energy * se;
                        out[s] = (OUT)(fma(sr, sr, si * si) / (den > 1e-12 ? den : 1e-12));
                    }
                }
                wave_sync();                                           // partials rewritten next round
            }
        }
        return;
    }
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


// ------------------------------------------------------------------------------------------------
// Pair kernel: the template bins come in pairs (k, N - k) (the ZC template's ±1 .. ±31).  One real-
// coefficient resonator per pair and branch carries both bins (sliding Goertzel): with θ = 2πk/N,
// c2 = 2 cos θ and the comb input d = x[s'+N] - x[s'],
//     g ← d + c2·g - h,   h ← g                       (g = s_n, h = s_{n-1}; 4 VALU per pair)
//     y± = g - e^{∓iθ} h  = w^{±k} X_s[±k]             (the two bins, up to a constant phase)
// so per pair and offset:
//     numerator   conj(t+) X[k] + conj(t-) X[-k] = A·Σ_br g + B·Σ_br h     (8 FMA)
//     energy      |X[k]|² + |X[-k]|² = 2(|g|² + |h|² - c2·Re(g h*))          (|h|² = last step's |g|²)
// 17 VALU per pair and offset against 24 for the two bins' first-order recursions (12 each).  The
// resonator's poles e^{±iθ} stay on the unit circle in floating point (the constant term is exactly
// 1), so rounding only shifts θ by ~ε/sin θ; an error injected into g reaches y with gain 1, and the
// energy's cancellation costs ~ε/sin²θ relative (1e-11 at N = 2048, k = 1).  The plan requires
// sin θ >= 1/2048 for every pair.  Each chunk starts from its exact window (block sums, as above):
// h = -i(y+ - y-)/(2 sin θ), g = y+ + e^{-iθ} h.
// Lanes: a row of LPC = 32/PPL lanes per chunk, PPL pairs per lane (pair p = sl + LPC·q); pair slots
// past npairs have dm = 0 (their d is dropped), so their state stays 0.
template <int FMT, int NB, int PPL, class OUT, bool DEFER>
__global__ __launch_bounds__(64 * ZS_MAXW) void zc_pair_kernel(ZsArgs a) {
    constexpr int LPC = 32 / PPL;                                      // lanes per chunk row
    constexpr int ROWS = 64 / LPC;                                     // chunks per wave
    extern __shared__ __attribute__((aligned(16))) double2 zsm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int W = a.W, C = a.C, N = a.N, NQ = N / C;
    const int STG = zs_stg(C, ROWS);                                   // per-wave staging per branch
    const int64_t b = blockIdx.x / a.groups, gi = blockIdx.x - b * a.groups;
    const int64_t c0 = gi * ROWS * (int64_t)W;
    const int64_t c1 = min(c0 + ROWS * (int64_t)W, a.nchunks);
    const int nblk = (int)(c1 - c0) + NQ - 1;
    // Blocks of ONE branch at a time (NBB = 1 row of 64 slots per block): the branch's initial windows
    // are built from them before the next branch's blocks overwrite the region, so the workgroup's LDS
    // holds one branch's blocks (two branches: half the LDS, twice the resident workgroups)
    constexpr int NBB = 1;
    double2* beta = zsm;                                               // [nblk][NBB][64]
    double2* stg = zsm + (size_t)(ROWS * W + NQ - 1) * NBB * 64 + (size_t)w * zs_pair_stgw(C, ROWS, NB);

    const int row = lane / LPC, sl = lane % LPC;
    const int64_t c = c0 + ROWS * (int64_t)w + row;
    const bool idle = c0 + ROWS * (int64_t)w >= c1;
    const bool live = c < c1;
    const int cl = live ? (int)(c - c0) : 0;
    double2 g[PPL][NB], h[PPL][NB];
    double epp = 0.0;                                                  // Σ |h|² (last step's Σ |g|²)
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        if (rb > 0) __syncthreads();                                   // the previous branch's blocks are read
        if (a.gblk)
            zs_blocks_pair<FMT, NBB>(a, beta, stg, zs_stg(C, ROWS), b * NB + rb, c0, nblk, lane, w);
        else
            zs_blocks<FMT, NBB>(a, beta, stg, zs_stg(C, ROWS), b * NB + rb, c0, nblk, lane, w);
        __syncthreads();
        // branch rb's initial windows: X_s[±k] = Σ_{q<N/C} w^{±kqC} β_{±k}(c + q)
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const int p = sl + LPC * q;
            const bool valid = p < a.npairs && !idle;
            const int k = valid ? a.pk[p] : 1, sp = valid ? a.ps[p] : 0, sn = valid ? a.pn[p] : 0;
            const double2 w1 = twid(k, N);
            const double inv2s = -0.5 / w1.y;                          // 1 / (2 sin θ)
            const double2 step = twid(((int64_t)k * C) % N, N);        // w^{kC}
            double2 t = make_double2(1.0, 0.0), xp = make_double2(0.0, 0.0), xn = make_double2(0.0, 0.0);
            for (int pq = 0; pq < (valid ? NQ : 0); ++pq) {
                xp = cfma(t, beta[(cl + pq) * NBB * 64 + sp], xp);
                xn = cfma(make_double2(t.x, -t.y), beta[(cl + pq) * NBB * 64 + sn], xn);
                t = cmul(t, step);
            }
            const double2 yp = cmul(w1, xp), yn = cmul(make_double2(w1.x, -w1.y), xn);
            const double2 hh = make_double2((yp.y - yn.y) * inv2s, -(yp.x - yn.x) * inv2s);   // -i(y+ - y-)/(2 sin θ)
            const double2 gg = cfma(w1, hh, yp);
            h[q][rb] = valid ? hh : make_double2(0.0, 0.0);
            g[q][rb] = valid ? gg : make_double2(0.0, 0.0);
            epp = fma(h[q][rb].x, h[q][rb].x, fma(h[q][rb].y, h[q][rb].y, epp));
        }
    }
    if (!DEFER && idle) return;                                        // (no barrier follows)
    double c2[PPL], dm[PPL];
    double2 A[PPL], Bc[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
        const int p = sl + LPC * q;
        const bool valid = p < a.npairs && !idle;
        const int k = valid ? a.pk[p] : 1, sp = valid ? a.ps[p] : 0, sn = valid ? a.pn[p] : 0;
        const double2 w1 = twid(k, N);                                 // w^k = e^{-iθ}
        const double2 tp = make_double2(a.tr[sp], -a.ti[sp]), tn = make_double2(a.tr[sn], -a.ti[sn]);  // conj(t±)
        const double2 ap = cmul(tp, make_double2(w1.x, -w1.y)), an = cmul(tn, w1);
        A[q] = valid ? make_double2(ap.x + an.x, ap.y + an.y) : make_double2(0.0, 0.0);
        Bc[q] = valid ? make_double2(-(tp.x + tn.x), -(tp.y + tn.y)) : make_double2(0.0, 0.0);
        c2[q] = valid ? 2.0 * w1.x : 0.0;
        dm[q] = valid ? 1.0 : 0.0;
    }
    double2* dbuf = stg;                                               // [NB][ROWS][ZS_G]
    const int64_t o0 = c * (int64_t)C;
    OUT* out = static_cast<OUT*>(a.metric) + b * a.noff;
    // one offset: in-lane partials (numerator, energy) of the lane's pairs from (cur, prv) = (g, h)
    // or (h, g); the update writes the new g over prv, so two consecutive steps swap the roles of the
    // two register sets and no state is copied
    // sg[q] (two branches): the branch sum of the set that is `prv` in the coming step - a step's h
    // sums are the previous step's g sums, so each step forms only the g sums
    double2 sg[NB > 1 ? PPL : 1];
#pragma unroll
    for (int q = 0; q < (NB > 1 ? PPL : 0); ++q) {
        double sx = h[q][0].x, sy = h[q][0].y;
#pragma unroll
        for (int r = 1; r < NB; ++r) { sx += h[q][r].x; sy += h[q][r].y; }
        sg[q] = make_double2(sx, sy);
    }
    // e: HALF the energy (|g|² + |h|² - c2·Re(g h*) summed); the factor 2 sits in the denominator
    auto step_terms = [&](const double2 (&cur)[PPL][NB], const double2 (&prv)[PPL][NB], double& cr, double& ci,
                          double& e) {
        double ep = 0.0, ed = 0.0;
        cr = 0.0; ci = 0.0;
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            double gr = cur[q][0].x, gim = cur[q][0].y;
#pragma unroll
            for (int r = 1; r < NB; ++r) { gr += cur[q][r].x; gim += cur[q][r].y; }
            double hr = prv[q][0].x, him = prv[q][0].y;
            if constexpr (NB > 1) {
                hr = sg[q].x; him = sg[q].y;
                sg[q] = make_double2(gr, gim);
            }
            cr = fma(A[q].x, gr, fma(-A[q].y, gim, fma(Bc[q].x, hr, fma(-Bc[q].y, him, cr))));
            ci = fma(A[q].x, gim, fma(A[q].y, gr, fma(Bc[q].x, him, fma(Bc[q].y, hr, ci))));
            double t = cur[q][0].y * prv[q][0].y;                      // Σ_br Re(g h*)
            t = fma(cur[q][0].x, prv[q][0].x, t);
#pragma unroll
            for (int r = 1; r < NB; ++r) t = fma(cur[q][r].x, prv[q][r].x, fma(cur[q][r].y, prv[q][r].y, t));
#pragma unroll
            for (int r = 0; r < NB; ++r) ep = fma(cur[q][r].x, cur[q][r].x, fma(cur[q][r].y, cur[q][r].y, ep));
            ed = fma(c2[q], t, ed);
        }
        e = (ep + epp) - ed;
        epp = ep;
    };
    const double te2 = 2.0 * a.t_energy;                               // template energy x the energy's 2
    auto advance = [&](const double2 (&cur)[PPL][NB], double2 (&prv)[PPL][NB], int u) {
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            const double2 d = dbuf[(r * ROWS + row) * ZS_G + u];
#pragma unroll
            for (int q = 0; q < PPL; ++q) {
                const double2 tq = make_double2(fma(dm[q], d.x, -prv[q][r].x), fma(dm[q], d.y, -prv[q][r].y));
                prv[q][r] = make_double2(fma(c2[q], cur[q][r].x, tq.x), fma(c2[q], cur[q][r].y, tq.y));
            }
        }
    };
    if constexpr (DEFER) {
        __syncthreads();                                               // blocks dead: partials take their place
        if (idle) return;
        double* part = reinterpret_cast<double*>(zsm) + (size_t)w * (ZS_RG * ZS_PS);
        for (int og = 0; og < C; og += ZS_G) {
            zs_stage_d<FMT, NB, LPC, ROWS>(a, dbuf, b, o0, og, live, row, sl);
            wave_sync();
#pragma unroll 1
            for (int v = 0; v < ZS_G / ZS_RG; ++v) {
#pragma unroll 1
                for (int uu = 0; uu < ZS_RG; uu += 2) {
                    double cr, ci, e;
                    step_terms(g, h, cr, ci, e);
                    part[uu * ZS_PS + lane] = cr;
                    part[uu * ZS_PS + 64 + lane] = ci;
                    part[uu * ZS_PS + 128 + lane] = e;
                    advance(g, h, v * ZS_RG + uu);                     // h <- new state
                    step_terms(h, g, cr, ci, e);
                    part[(uu + 1) * ZS_PS + lane] = cr;
                    part[(uu + 1) * ZS_PS + 64 + lane] = ci;
                    part[(uu + 1) * ZS_PS + 128 + lane] = e;
                    advance(h, g, v * ZS_RG + uu + 1);                 // g <- new state
                }
                wave_sync();
                if (sl < ZS_RG) {                                      // lane (row, j): step v·RG + j
                    const double* pp = part + sl * ZS_PS + row * LPC;
                    double sr = 0.0, si = 0.0, se = 0.0;
#pragma unroll
                    for (int l = 0; l < LPC; l += 2) {
                        const double2 pr = *reinterpret_cast<const double2*>(pp + l);
                        const double2 pi = *reinterpret_cast<const double2*>(pp + 64 + l);
                        const double2 pe = *reinterpret_cast<const double2*>(pp + 128 + l);
                        sr += pr.x + pr.y;
                        si += pi.x + pi.y;
                        se += pe.x + pe.y;
                    }
                    const int64_t s = o0 + og + v * ZS_RG + sl;
                    if (live && s < a.noff) {
                        const double den = te2 * se;
                        out[s] = (OUT)(fma(sr, sr, si * si) / (den > 1e-12 ? den : 1e-12));
                    }
                }
                wave_sync();
            }
        }
        return;
    }
    // steps u, u + 1 reduced together (row_sum2): the lower half of the row ends with step u, the upper
    // half with u + 1, so lane (hi, pos) keeps the steps 2(pos + HALF·j) + hi of the group
    // STEPS consecutive steps reduced together (row_sum2 / row_sum4): lane (which, pos) of the row ends
    // with step u + which and keeps the steps STEPS·(pos + SPAN·j) + which of the group
    constexpr int STEPS = LPC == 16 ? 4 : 2, SPAN = LPC / STEPS, KEEP = ZS_G / LPC;
    const int which = sl / SPAN, pos = sl % SPAN;
    for (int og = 0; og < C; og += ZS_G) {
        zs_stage_d<FMT, NB, LPC, ROWS>(a, dbuf, b, o0, og, live, row, sl);
        wave_sync();
        double keep_n[KEEP], keep_e[KEEP];
#pragma unroll
        for (int j = 0; j < KEEP; ++j) { keep_n[j] = 0.0; keep_e[j] = 0.0; }
#pragma unroll 1
        for (int u = 0; u < ZS_G; u += STEPS) {
            double cr, ci, e;
            if constexpr (STEPS == 4) {
                double cr0, ci0, e0, cr1, ci1, e1, cr2, ci2, e2, cr3, ci3, e3;
                step_terms(g, h, cr0, ci0, e0);
                advance(g, h, u);
                step_terms(h, g, cr1, ci1, e1);
                advance(h, g, u + 1);
                step_terms(g, h, cr2, ci2, e2);
                advance(g, h, u + 2);
                step_terms(h, g, cr3, ci3, e3);
                advance(h, g, u + 3);
                cr = row_sum4(cr0, cr1, cr2, cr3);
                ci = row_sum4(ci0, ci1, ci2, ci3);
                e = row_sum4(e0, e1, e2, e3);
            } else {
                double cr0, ci0, e0, cr1, ci1, e1;
                step_terms(g, h, cr0, ci0, e0);
                advance(g, h, u);
                step_terms(h, g, cr1, ci1, e1);
                advance(h, g, u + 1);
                cr = row_sum2<LPC>(cr0, cr1);
                ci = row_sum2<LPC>(ci0, ci1);
                e = row_sum2<LPC>(e0, e1);
            }
            const double n2 = fma(cr, cr, ci * ci);
#pragma unroll
            for (int j = 0; j < KEEP; ++j)
                if (u / STEPS == pos + SPAN * j) { keep_n[j] = n2; keep_e[j] = e; }
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < KEEP; ++j) {
            const int64_t s = o0 + og + STEPS * (pos + SPAN * j) + which;
            if (live && s < a.noff) {
                const double den = te2 * keep_e[j];
                out[s] = (OUT)(keep_n[j] / (den > 1e-12 ? den : 1e-12));
            }
        }
    }
}

}  // namespace

namespace {
// Row sums: deferred LDS partials for one branch, per-step DPP for two (measured, profiles/r03l_*:
// one branch 0.188 -> 0.183 ms, two branches 0.796 -> 0.840 ms); variant ZS_DEFER=0|1 forces either (A/B)
bool zs_defer(int n_br) {
    const int64_t v = ofs::variant(ofs::V_ZS_DEFER);
    return v != INT64_MIN ? v != 0 : n_br == 1;
}

// variant ZS_PAIR=0: the per-bin kernel even for a paired template (A/B)
bool zs_pair_enabled() {
    return !ofs::variant_off(ofs::V_ZS_PAIR);
}

template <class K>
int zs_launch(K kern, bool& attr, const ZsArgs& a, size_t lds, hipStream_t st) {
    if (!attr) {                                      // the dynamic-LDS limit, once per instantiation
        if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return OFS_EHIP;
        attr = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)(a.B * a.groups)), dim3(64 * a.W), lds, st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

template <int FMT, int NB, class OUT>
int zs_go(const ZsArgs& a, size_t lds, int bpl, bool pair, hipStream_t st) {
    bool df = zs_defer(NB);
    // the pair kernel parks the waves' partials in its block region (one branch's blocks): where
    // they would reach past it into the waves' staging, the per-step DPP row sums serve instead
    if (pair && df && (size_t)a.W * ZS_RG * ZS_PS * sizeof(double) >
                          (size_t)(bpl * a.W + a.N / a.C - 1) * 64 * sizeof(double2))
        df = false;
    static bool at[6] = {false, false, false, false, false, false};
    if (pair) {
        constexpr int PPL = NB == 2 ? 2 : 4;          // rows of 32/PPL lanes: 4 chunks (two branches) / 8 per wave
        return df ? zs_launch(zc_pair_kernel<FMT, NB, PPL, OUT, true>, at[0], a, lds, st)
                  : zs_launch(zc_pair_kernel<FMT, NB, PPL, OUT, false>, at[1], a, lds, st);
    }
    if constexpr (NB == 2) {
        return df ? zs_launch(zc_slide_kernel<FMT, 2, 4, OUT, true>, at[2], a, lds, st)
                  : zs_launch(zc_slide_kernel<FMT, 2, 4, OUT, false>, at[3], a, lds, st);
    } else {
        if (bpl == 4)                                 // 4 one-branch bins per lane: the block region
            return zs_launch(zc_slide_kernel<FMT, 1, 4, OUT, false>, at[4], a, lds, st);   // may not hold the partials
        return df ? zs_launch(zc_slide_kernel<FMT, 1, 8, OUT, true>, at[2], a, lds, st)
                  : zs_launch(zc_slide_kernel<FMT, 1, 8, OUT, false>, at[3], a, lds, st);
    }
}

// The pair kernel's template condition: every bin pairs with its mirror N - k (neither 0 nor N/2)
// and sin(2πk/N) >= 1/2048 (the resonator's error grows as 1/sin θ).  Fills a.npairs / pk / ps / pn.
bool zs_pairs(ZsArgs& a) {
    const int N = a.N, n = a.nbins;
    if (n % 2 || n > 64) return false;
    bool used[64] = {};
    int np = 0;
    for (int i = 0; i < n; ++i) {
        const int k = a.kb[i];
        if (k <= 0 || 2 * k == N || k >= N) return false;
        if (2 * k > N) continue;                      // the mirror half is matched from its partner
        int j = -1;
        for (int m = 0; m < n; ++m)
            if (!used[m] && m != i && a.kb[m] == N - k) { j = m; break; }
        if (j < 0 || used[i]) return false;
        if (std::sin(2.0 * M_PI * k / N) < 1.0 / 2048) return false;
        used[i] = used[j] = true;
        a.pk[np] = k; a.ps[np] = i; a.pn[np] = j;
        ++np;
    }
    if (2 * np != n) return false;
    a.npairs = np;
    for (int p = np; p < 32; ++p) { a.pk[p] = 1; a.ps[p] = 0; a.pn[p] = 0; }
    return true;
}
}  // namespace

namespace {
// chunk / block length C (C | N; 256 for N >= 8192 keeps the blocks per window at <= 32), waves per
// workgroup W (<= 16; 8 for two branches) and the workgroup's LDS; false if the blocks do not fit
// bins per lane of the slide: 8 for one branch (variant ZS_BPL=4 for the A/B), 4 for two (8 would
// exceed the 128 VGPRs of a 16-wave workgroup and spill)
int zs_bpl(int n_br) {
    return (n_br == 2 || ofs::variant_is(ofs::V_ZS_BPL, 4)) ? 4 : 8;
}

bool zs_plan(int n_br, int N, int bpl, int& C, int& W, size_t& lds, int64_t noff) {
    C = (N >= 8192 && N % 256 == 0) ? 256 : (N % 128 == 0 ? 128 : 64);
    {                                                                  // A/B: chunk length override
        const int64_t c = ofs::variant(ofs::V_ZS_C);
        if (c >= 64 && c <= 256 && c % 64 == 0 && N % c == 0) C = (int)c;
    }
    const int64_t nchunks = (noff + C - 1) / C;
    W = (int)std::min<int64_t>(n_br == 1 ? 16 : 8, (nchunks + bpl - 1) / bpl);
    const int stg = zs_stg(C, bpl);
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
    a.npairs = 0;
    a.gblk = !ofs::variant_off(ofs::V_ZS_GBLK);                     // 0: Horner block DFTs in the pair kernel (A/B)
    const bool pair = zs_pair_enabled() && bpl == (n_br == 2 ? 4 : 8) && zs_pairs(a);
    if (pair) lds = zs_pair_lds(a.C, N, bpl, a.W, n_br);        // one branch's blocks at a time
#define ZS_CASE(F, NBV) \
    if (fmt == F && n_br == NBV) \
        return f ? zs_go<F, NBV, float>(a, lds, bpl, pair, st) : zs_go<F, NBV, double>(a, lds, bpl, pair, st);
    ZS_CASE(OFS_C64, 1) ZS_CASE(OFS_C64, 2) ZS_CASE(OFS_C128, 1) ZS_CASE(OFS_C128, 2)
    ZS_CASE(OFS_CI16, 1) ZS_CASE(OFS_CI16, 2)
#undef ZS_CASE
    return 0;
}
