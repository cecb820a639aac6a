// zc_fftcorr.hip — the ZC matched filter through FFT overlap-save (SURVEY §8(f)3 "via FFT
// correlation"): np.convolve(x, conj(ref[::-1]), 'full') of zc_v2.py:244-254 / zc.py:115-126
// with a 2048-tap reference costs 2048 complex MACs per output as a direct sum (corr.hip,
// zc_mf_kernel: fp64 vector-FMA bound); as overlap-save it is a few FFT passes per output.
//
//   block q of a row: u_q[m] = xz[q·S - (N-1) + m], m in [0, M)  (xz: x zero-padded), S = M - N + 1
//   U = FFT_M(u_q) · H,  H = FFT_M(h),  h[i] = conj(ref[N-1-i]) zero-padded   (rocFFT, fp64)
//   corr[q·S + s] = IFFT_M(U)[N - 1 + s] / M,  s in [0, S)
//
// Kernels: pack (rows x blocks into a [rows·nblk][M] c128 scratch), rocFFT forward (in place),
// pointwise ·H, rocFFT inverse (in place), extract: per (stream, block) one workgroup reads the
// valid part of every branch, combines the branches as the modes of ofs_zc_correlate (raw /
// zc_v2 detect combine / zc.py combine / sum) and normalises with the sliding window energy
// Σ|x|² over the same N samples, from an fp64 prefix scan of |u_q|² in LDS (error relative to
// the block's energy, M = 4N samples).
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>
#include <stdint.h>
#include <math.h>
#include <mutex>
#include <algorithm>
#include <cstdlib>
#include "ofdmsync.h"
#include "ofs_common.h"

namespace {

constexpr int FW = 256;
#ifndef OFS_MC_FX
#define OFS_MC_FX 1024
#endif
constexpr int FX = OFS_MC_FX;     // extract workgroup (energy prefix + normalised outputs)

struct McPlan {
    rocfft_plan fwd = nullptr, inv = nullptr;
    int32_t N = 0, M = 0, S = 0, nb = 0;
    int64_t B = 0, T = 0, nblk = 0, nout = 0;
    double2* H = nullptr;           // [M] FFT of the reversed conjugated reference
    double2* Hbr = nullptr;         // fused path (M = MF_M): H[bitrev(i)] / M, then 128 twiddles
    double ref_norm = 0.0;
    int n_cu = 0;                   // persistent fused kernel: workgroups (one per CU), 0 = not set up
    size_t work_bytes = 0;
    size_t scratch_bytes = 0;
    rocfft_execution_info info = nullptr;   // reused by every call (stream / work buffer set per call)
};

std::once_flag g_setup;

template <int FMT>
__device__ __forceinline__ double2 ldx(const void* x, int64_t i) {
    if constexpr (FMT == OFS_C64) {
        const float2 v = static_cast<const float2*>(x)[i];
        return make_double2(v.x, v.y);
    } else if constexpr (FMT == OFS_C128) {
        return static_cast<const double2*>(x)[i];
    } else {
        const short2 v = static_cast<const short2*>(x)[i];
        return make_double2(v.x, v.y);
    }
}

struct McArgs {
    const void* x; int64_t T; int nb; int N, M, S; int64_t nblk, nout; int mode;
    double ref_norm; double2* U; const double2* H; double2* out; double* mag;
};

// U[(row·nblk + q)][m] = xz_row[q·S - (N-1) + m]
template <int FMT>
__global__ __launch_bounds__(FW) void mc_pack_kernel(McArgs a) {
    const int64_t blk = blockIdx.y;                 // row·nblk + q
    const int64_t row = blk / a.nblk, q = blk - row * a.nblk;
    const int64_t g0 = q * a.S - (a.N - 1);
    double2* dst = a.U + blk * a.M;
    for (int m = blockIdx.x * FW + threadIdx.x; m < a.M; m += gridDim.x * FW) {
        const int64_t g = g0 + m;
        dst[m] = (g >= 0 && g < a.T) ? ldx<FMT>(a.x, row * a.T + g) : make_double2(0.0, 0.0);
    }
}

// U *= H / M (pointwise, every block)
__global__ __launch_bounds__(FW) void mc_mul_kernel(double2* U, const double2* H, int64_t n, int M, double scale) {
    for (int64_t i = blockIdx.x * (int64_t)FW + threadIdx.x; i < n; i += (int64_t)gridDim.x * FW) {
        const double2 u = U[i], h = H[i % M];
        U[i] = make_double2((u.x * h.x - u.y * h.y) * scale, (u.x * h.y + u.y * h.x) * scale);
    }
}

// ---- fused overlap-save block (M = MF_M = 8192): pack + FFT + ·H/M + inverse FFT in one kernel ----
// One 1024-thread workgroup per (row, block), the block in LDS (128 KiB), never in HBM between the
// transforms (the rocFFT path writes and reads the [rows·nblk][M] scratch four times, plus pack and
// multiply passes).  Forward: decimation in frequency, natural order in -> bit-reversed order out, so
// the pointwise product uses H in bit-reversed order (Hbr, built with the plan) and needs no
// reordering; inverse = conj(DFT(conj(·))), a decimation-in-time DFT: bit-reversed in -> natural out.
// Thread t holds samples t + 1024·m (m < 8): the three largest-span stages of each transform run in
// registers (the load / the final store), the other ten as radix-8, radix-8, radix-4, radix-4 LDS
// passes.  Twiddles w^j (w = e^{-2 pi i/M}) from two 64-entry LDS tables; the block sits in LDS with
// one pad per 16 elements (141 KiB per workgroup).  Only the valid outputs m >= N-1 are written to
// the scratch the extract kernel reads.  512 x 16384 c128, 2048 taps: pack + rocFFT + multiply +
// rocFFT (~305 us) -> 160-173 us; the whole matched filter 0.52 -> 0.37 ms (profiles/r03z*).
constexpr int MF_T = 1024;
#ifndef OFS_MC_MID16
#define OFS_MC_MID16 1          // the transforms' middle (spans 8..1, xH, 1..8) as one 16-element pass
#endif
constexpr int MF_M = 8 * MF_T;

// twiddle w^e, e < M/2, from two 64-entry LDS tables: w^e = w^{64·(e>>6)} · w^{e & 63} (one complex
// product, ~1 ulp more than a full table; the full quarter table would not fit beside the block)
__device__ __forceinline__ double2 mf_tw(const double2* tws, int e) {
    const double2 a = tws[64 + (e >> 6)], b = tws[e & 63];
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// LDS slot (16 B) of block element e: its low four bits XORed with bits 3-6 (a bijection: the high bits
// fix bit 3's partner first).  ds_read_b128 services a wave in four 16-lane groups of one 256-B bank
// row each ({0-3,12-15,20-27}, ...: MI355X_MICROARCH.md §LDS) and ds_write_b128 in eight groups of 8
// contiguous lanes; for every access of this kernel - elements t + 1024m, the radix-8 groups at spans
// 128 and 16, the lane-pair 16-groups 8t + i - the slots of a group are then distinct (modelled: 0
// extra cycles; the earlier one-pad-per-16 layout left 2-way conflicts in five of the seven accesses,
// SQ_LDS_BANK_CONFLICT 28 % of the LDS-active cycles, profiles/r04c_*)
__device__ __forceinline__ int mf_at(int e) { return e ^ ((e >> 3) & 15); }
// LDS position of the energy prefix P[j], j <= M (fused extract): one pad per 8 doubles, so a lane's
// eight consecutive prefixes (lanes 8 apart) hit 16 different slots of a ds_write_b64 group
__device__ __forceinline__ int mf_pq(int j) { return j + (j >> 3); }
constexpr int MF_LDS = (MF_M + 128) * 16;                 // block + the two twiddle tables
__device__ __forceinline__ double2 mf_mul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// w · e^{-i·pi·e8/4} for an eighth-turn count e8 in 0..3 known at compile time: the twiddles of one
// radix group differ from its base twiddle by such exact constants, so a group reads ONE table
// entry pair instead of one per butterfly (exponent (k + q·h)·M/(2·sp·h) = base^{R/(2sp)} · e^{-i·pi·q/sp})
__device__ __forceinline__ double2 mf_rot8(double2 w, int e8) {
    constexpr double r = 0.70710678118654752440;
    switch (e8) {
        case 0: return w;
        case 1: return make_double2(r * (w.x + w.y), r * (w.y - w.x));
        case 2: return make_double2(w.y, -w.x);
        default: return make_double2(r * (w.y - w.x), -r * (w.x + w.y));
    }
}
// the stage twiddle of butterfly q at half-span sp (in units of h) of a radix-R group whose powers of
// the base twiddle are pw[0] = b, pw[1] = b^2, pw[2] = b^4
template <int R>
__device__ __forceinline__ double2 mf_stw(const double2 (&pw)[3], int sp, int q) {
    const int pi = (R / (2 * sp)) == 1 ? 0 : ((R / (2 * sp)) == 2 ? 1 : 2);
    return mf_rot8(pw[pi], q * (4 / sp));
}
template <int R>
__device__ __forceinline__ void mf_powers(const double2* twq, int e, double2 (&pw)[3]) {
    pw[0] = mf_tw(twq, e);
    pw[1] = mf_mul(pw[0], pw[0]);
    if (R == 8) pw[2] = mf_mul(pw[1], pw[1]);
    else pw[2] = pw[1];
}
__device__ __forceinline__ void mf_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// DIF radix-R pass over spans (R/2)h .. h; LAST: then ·Hbr and conjugate (the inverse's input)
template <int R, bool LAST>
__device__ __forceinline__ void mf_dif(double2* fb, const double2* twq, int h, const double2* __restrict__ Hbr) {
    for (int j = threadIdx.x; j < MF_M / R; j += MF_T) {
        const int g = j / h, k = j - g * h;
        const int p = g * R * h + k;
        double2 v[R];
#pragma unroll
        for (int i = 0; i < R; ++i) v[i] = fb[mf_at(p + i * h)];
        double2 pw[3];
        mf_powers<R>(twq, k * (MF_M / (R * h)), pw);
#pragma unroll
        for (int sp = R / 2; sp >= 1; sp >>= 1) {
            double2 w[R / 2];
#pragma unroll
            for (int q = 0; q < sp; ++q) w[q] = mf_stw<R>(pw, sp, q);
#pragma unroll
            for (int i0 = 0; i0 < R; i0 += 2 * sp)
#pragma unroll
                for (int q = 0; q < sp; ++q) {
                    const double2 a = v[i0 + q], b = v[i0 + q + sp];
                    v[i0 + q] = make_double2(a.x + b.x, a.y + b.y);
                    v[i0 + q + sp] = mf_mul(make_double2(a.x - b.x, a.y - b.y), w[q]);
                }
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
            if (LAST) {
                const double2 y = mf_mul(v[i], Hbr[p + i * h]);
                v[i] = make_double2(y.x, -y.y);
            }
            fb[mf_at(p + i * h)] = v[i];
        }
    }
    mf_sync();
}
// DIT radix-R pass over spans h .. (R/2)h
template <int R>
__device__ __forceinline__ void mf_dit(double2* fb, const double2* twq, int h) {
    for (int j = threadIdx.x; j < MF_M / R; j += MF_T) {
        const int g = j / h, k = j - g * h;
        const int p = g * R * h + k;
        double2 v[R];
#pragma unroll
        for (int i = 0; i < R; ++i) v[i] = fb[mf_at(p + i * h)];
        double2 pw[3];
        mf_powers<R>(twq, k * (MF_M / (R * h)), pw);
#pragma unroll
        for (int sp = 1; sp < R; sp <<= 1) {
            double2 w[R / 2];
#pragma unroll
            for (int q = 0; q < sp; ++q) w[q] = mf_stw<R>(pw, sp, q);
#pragma unroll
            for (int i0 = 0; i0 < R; i0 += 2 * sp)
#pragma unroll
                for (int q = 0; q < sp; ++q) {
                    const double2 t = mf_mul(w[q], v[i0 + q + sp]), u = v[i0 + q];
                    v[i0 + q] = make_double2(u.x + t.x, u.y + t.y);
                    v[i0 + q + sp] = make_double2(u.x - t.x, u.y - t.y);
                }
        }
#pragma unroll
        for (int i = 0; i < R; ++i) fb[mf_at(p + i * h)] = v[i];
    }
    mf_sync();
}

// v · e^{-i·pi·q/8}, q in 0..7 known at compile time (the 16th roots of unity of a radix-16 group at
// offset k = 0, whose twiddles are all constants)
__device__ __forceinline__ double2 mf_w16(double2 v, int q) {
    constexpr double c = 0.92387953251128675613, s = 0.38268343236508977173, r = 0.70710678118654752440;
    switch (q) {
        case 0: return v;
        case 1: return make_double2(v.x * c + v.y * s, v.y * c - v.x * s);
        case 2: return make_double2(r * (v.x + v.y), r * (v.y - v.x));
        case 3: return make_double2(v.x * s + v.y * c, v.y * s - v.x * c);
        case 4: return make_double2(v.y, -v.x);
        case 5: return make_double2(v.y * c - v.x * s, -(v.y * s + v.x * c));
        case 6: return make_double2(r * (v.y - v.x), -r * (v.x + v.y));
        default: return make_double2(v.y * s - v.x * c, -(v.y * c + v.x * s));
    }
}
// The middle of the matched filter in ONE LDS pass: the forward transform's last four DIF stages
// (spans 8, 4, 2, 1), the product with H/M in bit-reversed order and the conjugation, then the
// inverse's first four DIT stages (spans 1, 2, 4, 8) all act on the same 16 contiguous elements.  A
// lane pair holds one such group (lane t: elements 8t .. 8t+7, its partner t^1 the other half); the
// span-8 stages pair element i with i + 8 across the pair (DPP quad_perm [1,0,3,2] swap), spans 4..1
// stay inside a lane.  Every twiddle is a 16th root of unity (offset k = 0 in the group): constants.
// 1 LDS pass and barrier instead of 4, all 1024 threads busy.
__device__ __forceinline__ double2 mf_swap_pair(double2 v) {
    return make_double2(ofs::dpp_d<0xB1>(v.x), ofs::dpp_d<0xB1>(v.y));
}
__device__ __forceinline__ void mf_mid16(double2* fb, const double2* __restrict__ Hbr) {
    const int t = threadIdx.x;
    const bool hi = (t & 1) != 0;                   // elements 8..15 of the group
    double2 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fb[mf_at(8 * t + i)];
    // DIF span 8: a = element i, b = element i + 8 -> a + b (low half), (a - b)·w16^i (high half)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double2 o = mf_swap_pair(v[i]);
        const double2 a = hi ? o : v[i], b = hi ? v[i] : o;
        v[i] = hi ? mf_w16(make_double2(a.x - b.x, a.y - b.y), i) : make_double2(a.x + b.x, a.y + b.y);
    }
#pragma unroll
    for (int sp = 4; sp >= 1; sp >>= 1)
#pragma unroll
        for (int i0 = 0; i0 < 8; i0 += 2 * sp)
#pragma unroll
            for (int q = 0; q < sp; ++q) {
                const double2 a = v[i0 + q], b = v[i0 + q + sp];
                v[i0 + q] = make_double2(a.x + b.x, a.y + b.y);
                v[i0 + q + sp] = mf_w16(make_double2(a.x - b.x, a.y - b.y), q * (8 / sp));
            }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double2 y = mf_mul(v[i], Hbr[8 * t + i]);
        v[i] = make_double2(y.x, -y.y);
    }
#pragma unroll
    for (int sp = 1; sp <= 4; sp <<= 1)
#pragma unroll
        for (int i0 = 0; i0 < 8; i0 += 2 * sp)
#pragma unroll
            for (int q = 0; q < sp; ++q) {
                const double2 tt = mf_w16(v[i0 + q + sp], q * (8 / sp)), u = v[i0 + q];
                v[i0 + q] = make_double2(u.x + tt.x, u.y + tt.y);
                v[i0 + q + sp] = make_double2(u.x - tt.x, u.y - tt.y);
            }
    // DIT span 8: u = element i, w = w16^i · element i + 8 -> u + w (low half), u - w (high half)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double2 o = mf_swap_pair(v[i]);
        const double2 u = hi ? o : v[i], w = mf_w16(hi ? v[i] : o, i);
        v[i] = hi ? make_double2(u.x - w.x, u.y - w.y) : make_double2(u.x + w.x, u.y + w.y);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) fb[mf_at(8 * t + i)] = v[i];
    mf_sync();
}

template <int FMT, bool FUSE_X>
__global__ __launch_bounds__(MF_T) void mc_fused_kernel(McArgs a, const double2* __restrict__ Hbr) {
    extern __shared__ __attribute__((aligned(16))) double2 fb[];     // [MF_M + pads], then 2 x 64 twiddles
    const int t = threadIdx.x;
    double2* tws = fb + MF_M;
    if (t < 128) tws[t] = Hbr[MF_M + t];                              // w^l, l < 64; w^{64h}, h < 64 (plan)
    mf_sync();
    const double2* twq = tws;
    const int64_t blk = blockIdx.x;                                   // row·nblk + q
    const int64_t row = blk / a.nblk, q = blk - row * a.nblk;
    const int64_t g0 = q * a.S - (a.N - 1);
    double2 v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int64_t g = g0 + t + MF_T * m;
        v[m] = (g >= 0 && g < a.T) ? ldx<FMT>(a.x, row * a.T + g) : make_double2(0.0, 0.0);
    }
    // forward DIF, spans 4096, 2048, 1024 (twiddle exponents offset·M/(2·span)): with b = w^t,
    // w^{t + 1024m} = b·e^{-i pi m/4}, w^{2(t + 1024r)} = b^2·e^{-i pi r/2}, w^{4t} = b^4
    double2 tp[3];
    mf_powers<8>(twq, t, tp);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const double2 x0 = v[m], x1 = v[m + 4];
        v[m] = make_double2(x0.x + x1.x, x0.y + x1.y);
        v[m + 4] = mf_mul(make_double2(x0.x - x1.x, x0.y - x1.y), mf_rot8(tp[0], m));
    }
#pragma unroll
    for (int m = 0; m < 8; m += 4)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const double2 x0 = v[m + r], x1 = v[m + r + 2];
            v[m + r] = make_double2(x0.x + x1.x, x0.y + x1.y);
            v[m + r + 2] = mf_mul(make_double2(x0.x - x1.x, x0.y - x1.y), mf_rot8(tp[1], 2 * r));
        }
#pragma unroll
    for (int m = 0; m < 8; m += 2) {
        const double2 x0 = v[m], x1 = v[m + 1];
        v[m] = make_double2(x0.x + x1.x, x0.y + x1.y);
        v[m + 1] = mf_mul(make_double2(x0.x - x1.x, x0.y - x1.y), tp[2]);
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) fb[mf_at(t + MF_T * m)] = v[m];
    mf_sync();
    mf_dif<8, false>(fb, twq, 128, Hbr);                             // spans 512, 256, 128
    mf_dif<8, false>(fb, twq, 16, Hbr);                              // 64, 32, 16
#if OFS_MC_MID16
    mf_mid16(fb, Hbr);                                               // 8, 4, 2, 1; conj(X·H/M); 1, 2, 4, 8
#else
    mf_dif<4, false>(fb, twq, 4, Hbr);                               // 8, 4
    mf_dif<4, true>(fb, twq, 1, Hbr);                                // 2, 1; then conj(X·H/M)
    mf_dit<4>(fb, twq, 1);                                           // spans 1, 2
    mf_dit<4>(fb, twq, 4);                                           // 4, 8
#endif
    mf_dit<8>(fb, twq, 16);                                          // 16, 32, 64
    mf_dit<8>(fb, twq, 128);                                         // 128, 256, 512
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = fb[mf_at(t + MF_T * m)];
    // fused extract: the samples of the energy prefix (u[8t .. 8t+7], L2-resident) are requested now,
    // so their latency hides behind the inverse's last three register stages
    double2 u8[FUSE_X ? 8 : 1];
    if constexpr (FUSE_X) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int64_t g = g0 + 8 * t + i;
            u8[i] = (g >= 0 && g < a.T) ? ldx<FMT>(a.x, row * a.T + g) : make_double2(0.0, 0.0);
        }
    }
    mf_powers<8>(twq, t, tp);            // recomputed here rather than held across the LDS passes
#pragma unroll
    for (int m = 0; m < 8; m += 2) {                                 // span 1024
        const double2 tt = mf_mul(tp[2], v[m + 1]), u = v[m];
        v[m] = make_double2(u.x + tt.x, u.y + tt.y);
        v[m + 1] = make_double2(u.x - tt.x, u.y - tt.y);
    }
#pragma unroll
    for (int m = 0; m < 8; m += 4)                                   // span 2048
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const double2 tt = mf_mul(mf_rot8(tp[1], 2 * r), v[m + r + 2]), u = v[m + r];
            v[m + r] = make_double2(u.x + tt.x, u.y + tt.y);
            v[m + r + 2] = make_double2(u.x - tt.x, u.y - tt.y);
        }
#pragma unroll
    for (int m = 0; m < 4; ++m) {                                    // span 4096
        const double2 tt = mf_mul(mf_rot8(tp[0], m), v[m + 4]), u = v[m];
        v[m] = make_double2(u.x + tt.x, u.y + tt.y);
        v[m + 4] = make_double2(u.x - tt.x, u.y - tt.y);
    }
    if (!FUSE_X) {
        double2* dst = a.U + blk * (int64_t)MF_M;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int o = t + MF_T * m;
            if (o >= a.N - 1) dst[o] = make_double2(v[m].x, -v[m].y);   // conj: the inverse transform
        }
        return;
    }
    // ---- one branch: the extract fused in (mc_extract_kernel's arithmetic) ----
    // window energies from an fp64 prefix of |u_q|^2 over the block, in the (now free) block LDS:
    // thread t scans u[8t .. 8t+7] (re-read, L2), block scan of the thread totals, P[j] = Σ_{i<j}
    mf_sync();
    // P[j] lives at mf_pq(j) = j + j/8 (the plain layout [8t + i] put lanes 4 apart on one bank: 16-way
    // conflicts on the prefix stores, SQ_LDS_BANK_CONFLICT, profiles/r04b_*)
    double* P = reinterpret_cast<double*>(fb);                      // mf_pq(M) + 1 (+ per-wave totals)
    double* wt = P + MF_M + MF_M / 8 + 1;
    double e8[8], loc = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double e = u8[i].x * u8[i].x + u8[i].y * u8[i].y;     // 0 outside the stream (zero-filled)
        e8[i] = e;
        loc += e;
    }
    const int lane = t & 63, wv = t >> 6;
    double incl = loc;                                               // wave inclusive scan of the totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o2 = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o2;
    }
    if (lane == 63) wt[wv] = incl;
    mf_sync();
    double run = incl - loc;
    for (int k = 0; k < wv; ++k) run += wt[k];
    if (t == 0) P[mf_pq(0)] = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) { run += e8[i]; P[mf_pq(8 * t + i + 1)] = run; }
    mf_sync();
    const int64_t n0 = q * a.S;
    const int ns = (int)min((int64_t)a.S, a.nout - n0);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int o = t + MF_T * m, s = o - (a.N - 1);
        if (s < 0 || s >= ns) continue;
        const double2 c = make_double2(v[m].x, -v[m].y);
        const int64_t oi = row * a.nout + n0 + s;                    // one branch: row = stream
        // |.| as sqrt(re² + im²) and the normalisation as one reciprocal and two products: within an
        // ulp or two of numpy's hypot and true division (the block FFT's own error is ~1e-14 of the
        // row), without hypot's scaling branches and two fp64 divisions per output
        if (a.mode == OFS_ZC_RAW || a.mode == OFS_ZC_SUM) {
            if (a.out) a.out[oi] = c;
            if (a.mag) a.mag[oi] = sqrt(fma(c.x, c.x, c.y * c.y));
            continue;
        }
        const double e = P[mf_pq(o + 1)] - P[mf_pq(o + 1 - a.N)];  // Σ |x|^2 over the N-sample window
        const double ew = a.mode == OFS_ZC_V2 ? (e > 1e-12 ? e : 1e-12)                 // zc_v2.py:268
                                              : (e > 0.0 ? e : 0.0) + 1e-12;            // zc.py:113-126
        const double inv = 1.0 / (a.ref_norm * sqrt(ew));
        const double2 r = make_double2(c.x * inv, c.y * inv);
        if (a.out) a.out[oi] = r;
        if (a.mag) a.mag[oi] = sqrt(fma(r.x, r.x, r.y * r.y));
    }
}

// ---- persistent overlap-save kernel (M = 8192): one 512-thread workgroup per CU walks a contiguous run of
// blocks and overlaps each block's HBM traffic with the neighbouring blocks' arithmetic ----
// mc_fused_kernel runs one block per 1024-thread workgroup; its 141 KiB of LDS admit one workgroup per CU,
// so a block's 128 KiB input load, its FFTs and its 147 KiB of output stores run one after another on
// the CU (53 % of wave cycles waiting, 12.9 % VALU, profiles/r04d_*).  Here the next block's input is
// loaded into registers during the current block's second half, and the current block's stores drain
// during the next block's first half.  512 threads x 16 elements (2 waves per SIMD, up to 256 VGPRs):
//   forward DIF  spans 4096..512 in registers (elements t + 512m)    | twiddle base w_8192^t
//                spans  256..32  LDS pass, elements 512g + 32i + k    | base w_512^k  (g = t/32, k = t%32)
//                spans   16..1   LDS pass, elements 16t + i, lane pairs (span 16 across the pair by DPP)
//   conj(X * H / M) in bit-reversed order (Hbr, as mc_fused_kernel)
//   inverse DIT  spans 1..16 (same pass), 32..256 (LDS pass), 512..4096 (registers)
// 4 LDS passes instead of 5, two of them wave-local (no workgroup barrier), each stage's twiddle one
// product with a per-thread base (bases from a table built once per launch).  gfx9 counts loads and stores on one vmcnt, in issue
// order, so waiting for a load also waits for every store issued before it: the Hbr slice is loaded right after
// the previous block's stores (waited for in the middle pass, by when those stores have drained), and the
// next block's input is taken into registers BEFORE this block's stores are issued.
constexpr int MP_T = 512;
#ifndef OFS_MP_NTST
#define OFS_MP_NTST 1               // non-temporal output stores (measured 3-6 % faster, profiles/r05j_*)
#endif
#ifndef OFS_MP_CLAMPLOAD
#define OFS_MP_CLAMPLOAD 0
#endif
#ifndef OFS_MP_AB
#define OFS_MP_AB 0                 // diagnostic A/B builds only (wrong results): 1 no stores, 2 no sqrt/div,
#endif                              // 4 no energy prefix (the extract's LDS phase and its barriers), 8 no H loads
#ifndef OFS_MP_TIMING
#define OFS_MP_TIMING 0             // diagnostic builds: per-phase cycles of mc_pers_kernel (ofs_mp_prof)
#endif
#if OFS_MP_TIMING
__device__ unsigned long long mp_prof[8];
#endif
// LDS hand-over between the lanes of ONE wave: its LDS operations complete in order
#ifndef OFS_MP_WAVESYNC
#define OFS_MP_WAVESYNC 1           // tuning builds: 0 = workgroup barriers there as well
#endif
__device__ __forceinline__ void mp_wave_sync() {
#if OFS_MP_WAVESYNC
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#else
    mf_sync();
#endif
}
constexpr int MP_LDS = (MF_M + 512 + 32) * 16 + 8 * 8;   // block, w_8192^t (t < 512), w_512^k (k < 32), wave sums
// slot of block element e: low four bits XOR bits 4-7 (conflict-free for t + 512m, 512g + 32i + k, 16t + i)
__device__ __forceinline__ int mp_at(int e) { return e ^ ((e >> 4) & 15); }
typedef double mp_d2v __attribute__((ext_vector_type(2)));
#ifndef OFS_MP_ST16
#define OFS_MP_ST16 1               // 0: two 8-byte halves per complex output (A/B)
#endif
// energy prefix P[j] (doubles, in the block region during the extract): one pad per 16
__device__ __forceinline__ int mp_pq(int j) { return j + (j >> 4); }
__device__ __forceinline__ double2 c_add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 c_sub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
// v * e^{-i pi q / 16}, q < 16 known at compile time (the span-16 stage of the middle pass)
__device__ __forceinline__ double2 mp_w32(double2 v, int q) {
    if ((q & 1) == 0) return mf_w16(v, q >> 1);
    constexpr double C[8] = {0.98078528040323044913, 0.83146961230254523708, 0.55557023301960222474,
                             0.19509032201612826785, -0.19509032201612826785, -0.55557023301960222474,
                             -0.83146961230254523708, -0.98078528040323044913};   // cos(pi q / 16), q odd
    constexpr double S[8] = {0.19509032201612826785, 0.55557023301960222474, 0.83146961230254523708,
                             0.98078528040323044913, 0.98078528040323044913, 0.83146961230254523708,
                             0.55557023301960222474, 0.19509032201612826785};     // sin(pi q / 16)
    const double c = C[q >> 1], s = S[q >> 1];
    return make_double2(fma(v.x, c, v.y * s), fma(v.y, c, -(v.x * s)));
}
// 16-point radix-2 DIF over v[0..15] (spans 8, 4, 2, 1 in units of the caller's stride) with twiddles
// base^{j} * w16^{...}: span 8 pairs (m, m+8) take b * w16^m, span 4 b^2 * w16^{2(m%4)}, span 2
// b^4 * w16^{4(m%2)}, span 1 b^8.  UNIT: base 1 (no products with b).
template <bool UNIT>
__device__ __forceinline__ void mp_dif16(double2 (&v)[16], double2 b) {
    double2 b2 = b, b4 = b, b8 = b;
    if (!UNIT) { b2 = mf_mul(b, b); b4 = mf_mul(b2, b2); b8 = mf_mul(b4, b4); }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const double2 a = v[m], c = v[m + 8];
        v[m] = c_add(a, c);
        v[m + 8] = mf_w16(UNIT ? c_sub(a, c) : mf_mul(c_sub(a, c), b), m);
    }
#pragma unroll
    for (int h = 0; h < 16; h += 8)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const double2 a = v[h + m], c = v[h + m + 4];
            v[h + m] = c_add(a, c);
            v[h + m + 4] = mf_w16(UNIT ? c_sub(a, c) : mf_mul(c_sub(a, c), b2), 2 * m);
        }
#pragma unroll
    for (int h = 0; h < 16; h += 4)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const double2 a = v[h + m], c = v[h + m + 2];
            v[h + m] = c_add(a, c);
            v[h + m + 2] = mf_w16(UNIT ? c_sub(a, c) : mf_mul(c_sub(a, c), b4), 4 * m);
        }
#pragma unroll
    for (int m = 0; m < 16; m += 2) {
        const double2 a = v[m], c = v[m + 1];
        v[m] = c_add(a, c);
        v[m + 1] = UNIT ? c_sub(a, c) : mf_mul(c_sub(a, c), b8);
    }
}
// the matching radix-2 DIT (spans 1, 2, 4, 8): bit-reversed in, natural out
template <bool UNIT>
__device__ __forceinline__ void mp_dit16(double2 (&v)[16], double2 b) {
    double2 b2 = b, b4 = b, b8 = b;
    if (!UNIT) { b2 = mf_mul(b, b); b4 = mf_mul(b2, b2); b8 = mf_mul(b4, b4); }
#pragma unroll
    for (int m = 0; m < 16; m += 2) {
        const double2 u = v[m], w = UNIT ? v[m + 1] : mf_mul(v[m + 1], b8);
        v[m] = c_add(u, w);
        v[m + 1] = c_sub(u, w);
    }
#pragma unroll
    for (int h = 0; h < 16; h += 4)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const double2 u = v[h + m], w = mf_w16(UNIT ? v[h + m + 2] : mf_mul(v[h + m + 2], b4), 4 * m);
            v[h + m] = c_add(u, w);
            v[h + m + 2] = c_sub(u, w);
        }
#pragma unroll
    for (int h = 0; h < 16; h += 8)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const double2 u = v[h + m], w = mf_w16(UNIT ? v[h + m + 4] : mf_mul(v[h + m + 4], b2), 2 * m);
            v[h + m] = c_add(u, w);
            v[h + m + 4] = c_sub(u, w);
        }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const double2 u = v[m], w = mf_w16(UNIT ? v[m + 8] : mf_mul(v[m + 8], b), m);
        v[m] = c_add(u, w);
        v[m + 8] = c_sub(u, w);
    }
}

// 1/sqrt(x) for normal x > 0: v_rsq_f64 and two Newton steps y(1.5 - x y^2/2)
__device__ __forceinline__ double mp_rsqrt(double x) {
    double y = __builtin_amdgcn_rsq(x);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const double h = x * y;
        y = fma(0.5 * y, fma(-h, y, 1.0), y);
    }
    return y;
}
// sqrt(x), x >= 0: x rsqrt(x) for normal x, the library sqrt below 2^-1000 (0 and denormals)
__device__ __forceinline__ double mp_sqrt(double x) {
    if (x < 0x1p-1000) return sqrt(x);
    return x * mp_rsqrt(x);
}
// |c| (np.abs): mp_sqrt of |c|^2, or hypot where |c|^2 overflows (|c| > ~1.3e154: rsqrt(inf) = 0 would
// give inf·0 = NaN; numpy's hypot stays finite) or is NaN
__device__ __forceinline__ double mp_cabs(double2 c) {
    const double x = fma(c.x, c.x, c.y * c.y);
    if (!(x <= 0x1.fffffffffffffp+1023)) return hypot(c.x, c.y);
    return mp_sqrt(x);
}

// a block's samples t + 512m (zero outside the stream)
template <int FMT>
__device__ __forceinline__ void mp_load(const McArgs& a, int64_t row, int64_t q, int t, double2 (&d)[16]) {
    const int64_t g0 = q * a.S - (a.N - 1) + t;
    const int64_t base = row * a.T;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int64_t g = g0 + MP_T * m;
#if OFS_MP_CLAMPLOAD                // tuning builds: every lane loads a clamped in-stream index, then selects
        const bool in = g >= 0 && g < a.T;
        const double2 w = ldx<FMT>(a.x, base + (in ? g : 0));
        d[m] = in ? w : make_double2(0.0, 0.0);
#else
        d[m] = (g >= 0 && g < a.T) ? ldx<FMT>(a.x, base + g) : make_double2(0.0, 0.0);
#endif
    }
}

template <int FMT, bool FUSE_X>
__global__ __launch_bounds__(MP_T) void mc_pers_kernel(McArgs a, const double2* __restrict__ Hbr, int64_t total) {
    extern __shared__ __attribute__((aligned(16))) double2 fb[];    // [MF_M] block, tb[512], tc[32], wave sums
    double2* tb = fb + MF_M;
    double2* tc = tb + MP_T;
    double* wsum = reinterpret_cast<double*>(tc + 32);
    const int t0 = threadIdx.x, lane = t0 & 63, wv = t0 >> 6;
    {                                                               // twiddle bases, once per launch
        double sn, cs;
        sincospi(-2.0 * (double)t0 / (double)MF_M, &sn, &cs);
        tb[t0] = make_double2(cs, sn);                                // w_8192^t
        if (t0 < 32) {
            sincospi(-2.0 * (double)t0 / 512.0, &sn, &cs);
            tc[t0] = make_double2(cs, sn);                            // w_512^k
        }
    }
    const int64_t G = gridDim.x, wg = blockIdx.x;
    const int64_t b0 = wg * total / G, b1 = (wg + 1) * total / G;   // this workgroup's run of blocks
    const double rn_inv = 1.0 / a.ref_norm;
    if (b0 >= b1) return;                                           // (whole workgroup)
    double2 v[16];
    double en[FUSE_X ? 16 : 1];                                     // |u|^2 of this block's samples t + 512m
    int64_t row = b0 / a.nblk, q = b0 - (b0 / a.nblk) * a.nblk;   // block b0 = row * nblk + q (then stepped)
    mp_load<FMT>(a, row, q, t0, v);
    if constexpr (FUSE_X) {
#pragma unroll
        for (int m = 0; m < 16; ++m) en[m] = fma(v[m].x, v[m].x, v[m].y * v[m].y);
    }
#if OFS_MP_TIMING
    unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tl = __builtin_readcyclecounter();
#define MP_T_MARK(i) do { const unsigned long long tn = __builtin_readcyclecounter(); tacc[i] += tn - tl; tl = tn; } while (0)
#else
#define MP_T_MARK(i) do { } while (0)
#endif
#if OFS_MP_AB & 1
    const bool st_ok = a.T < 0;                                     // diagnostic: no stores
#else
    constexpr bool st_ok = true;
#endif
    for (int64_t blk = b0; blk < b1; ++blk) {
        if (blk > b0 && ++q == a.nblk) { q = 0; ++row; }          // (no 64-bit division per block)
        const int64_t nq = q + 1 == a.nblk ? 0 : q + 1, nrow = nq == 0 ? row + 1 : row;   // the next block
        // the thread index re-materialised per block (opaque to the optimiser): the per-thread LDS
        // addresses, twiddle bases and the H slice are loop-invariant, and hoisting them out of the block
        // loop would pin ~100 VGPRs for the whole launch
        int t = t0;
        asm volatile("" : "+v"(t));
        const int g2 = t >> 5, k2 = t & 31;                          // LDS pass position: 512 g2 + 32 i + k2
        // ---- forward: spans 4096..512 in registers ----
        mp_dif16<false>(v, tb[t]);
        MP_T_MARK(0);
        mf_sync();                                                  // previous block's LDS readers done
#pragma unroll
        for (int m = 0; m < 16; ++m) fb[mp_at(t + MP_T * m)] = v[m];
        mf_sync();
        MP_T_MARK(1);
        // ---- spans 256..32 ----
        {
            const int p = 512 * g2 + k2;
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = fb[mp_at(p + 32 * i)];
            mp_dif16<false>(v, tc[k2]);
#pragma unroll
            for (int i = 0; i < 16; ++i) fb[mp_at(p + 32 * i)] = v[i];
        }
        // spans 256..1 and back stay inside the 512 elements of group g2 = t / 32, which the half-wave t / 32
        // owns in this pass and the next: a wave-local hand-over, no workgroup barrier (the waves drift apart,
        // so one wave's LDS traffic overlaps another's arithmetic)
        mp_wave_sync();
        MP_T_MARK(2);
        // ---- spans 16..1, conj(X H / M), spans 1..16: lane pair (t, t^1) holds elements 32(t/2) .. +31 ----
        {
            const bool hi = (t & 1) != 0;
            // this block's H slice (L2-resident): waiting for it also waits for the previous block's stores
            // (one vmcnt), which have had the first two passes to drain
            double2 hb[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) hb[i] = (OFS_MP_AB & 8) ? make_double2(1.0, 0.0) : Hbr[16 * t + i];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = fb[mp_at(16 * t + i)];
#pragma unroll
            for (int i = 0; i < 16; ++i) {                          // DIF span 16 across the pair
                const double2 o = mf_swap_pair(v[i]);
                const double2 x0 = hi ? o : v[i], x1 = hi ? v[i] : o;
                v[i] = hi ? mp_w32(c_sub(x0, x1), i) : c_add(x0, x1);
            }
            mp_dif16<true>(v, make_double2(1.0, 0.0));
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const double2 y = mf_mul(v[i], hb[i]);
                v[i] = make_double2(y.x, -y.y);
            }
            mp_dit16<true>(v, make_double2(1.0, 0.0));
#pragma unroll
            for (int i = 0; i < 16; ++i) {                          // DIT span 16 across the pair
                const double2 o = mf_swap_pair(v[i]);
                const double2 u = hi ? o : v[i], w = mp_w32(hi ? v[i] : o, i);
                v[i] = hi ? c_sub(u, w) : c_add(u, w);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) fb[mp_at(16 * t + i)] = v[i];
        }
        mp_wave_sync();
        MP_T_MARK(3);
        // the next block's input: in flight through the second half of this block
        const bool more = blk + 1 < b1;
        double2 nx[16];
        if (more) {
            mp_load<FMT>(a, nrow, nq, t, nx);
        } else {
#pragma unroll
            for (int m = 0; m < 16; ++m) nx[m] = make_double2(0.0, 0.0);
        }
        // ---- inverse spans 32..256 ----
        {
            const int p = 512 * g2 + k2;
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = fb[mp_at(p + 32 * i)];
            mp_dit16<false>(v, tc[k2]);
#pragma unroll
            for (int i = 0; i < 16; ++i) fb[mp_at(p + 32 * i)] = v[i];
        }
        mf_sync();
        MP_T_MARK(4);
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = fb[mp_at(t + MP_T * m)];
        mp_dit16<false>(v, tb[t]);                                  // spans 512..4096: natural order out
        MP_T_MARK(5);
        const int64_t n0 = q * a.S;
        const int ns = (int)min((int64_t)a.S, a.nout - n0);
        if constexpr (!FUSE_X) {
#pragma unroll
            for (int m = 0; m < 16; ++m) { const double2 w = v[m]; v[m] = nx[m]; nx[m] = w; }   // next input in
            __builtin_amdgcn_sched_barrier(0);                      // ... before this block's stores
            double2* dst = a.U + blk * (int64_t)MF_M;
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int o = t + MP_T * m;
                if (o >= a.N - 1) dst[o] = make_double2(nx[m].x, -nx[m].y);
            }
            continue;
        }
        // ---- fused extract (one branch): window energies from an fp64 prefix of |u|^2 in the block LDS ----
        // P[j] = sum_{i<j} |u_i|^2 in place of |u_j|^2 (each thread rewrites only the 16 slots it read, so
        // no neighbour's input is overwritten), P[M] at slot mp_pq(M)
        double* P = reinterpret_cast<double*>(fb);
#if !(OFS_MP_AB & 4)
        mf_sync();                                                  // every thread has read its block slots
#pragma unroll
        for (int m = 0; m < 16; ++m) P[mp_pq(t + MP_T * m)] = en[m];
        mf_sync();
        double loc = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) loc += P[mp_pq(16 * t + i)];
        const double incl = ofs::wave_scan_add(loc, lane);
        if (lane == 63) wsum[wv] = incl;
        mf_sync();                                                  // (LDS re-read below: the fence)
        double run = incl - loc;
        for (int k = 0; k < wv; ++k) run += wsum[k];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int j = mp_pq(16 * t + i);
            const double e = P[j];
            P[j] = run;
            run += e;
        }
        if (t == MP_T - 1) P[mp_pq(MF_M)] = run;
#endif
        // next block's input taken into registers (and its energies) before any store of this block issues
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const double2 w = v[m];
            v[m] = nx[m];
            nx[m] = w;
            en[m] = fma(v[m].x, v[m].x, v[m].y * v[m].y);
        }
        mf_sync();
        MP_T_MARK(6);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const int o = t + MP_T * m, s = o - (a.N - 1);
            if (s < 0 || s >= ns) continue;
            const double2 c = make_double2(nx[m].x, -nx[m].y);
            const int64_t oi = row * a.nout + n0 + s;               // one branch: row = stream
            if (a.mode == OFS_ZC_RAW || a.mode == OFS_ZC_SUM) {
                if (a.out && st_ok) a.out[oi] = c;
                if (a.mag && st_ok) a.mag[oi] = mp_cabs(c);
                continue;
            }
#if OFS_MP_AB & 4
            const double e = 1.0 + en[m];
#else
            const double e = P[mp_pq(o + 1)] - P[mp_pq(o + 1 - a.N)];   // sum |x|^2 over the N-sample window
#endif
            const double ewc = a.mode == OFS_ZC_V2 ? (e > 1e-12 ? e : 1e-12)                 // zc_v2.py:268
                                                   : (e > 0.0 ? e : 0.0) + 1e-12;            // zc.py:113-126
            // 1 / (|ref| sqrt(e)) = rsqrt(e) / |ref| and |r| = s rsqrt(s), s = |r|^2: hardware rsqrt refined by
            // two Newton steps (an ulp or two from the reference's division and hypot, zc_v2.py:268-271)
            const double inv = mp_rsqrt(ewc) * rn_inv;
            const double2 r = make_double2(c.x * inv, c.y * inv);
#if OFS_MP_NTST                     // tuning builds: non-temporal output stores
            // (one 16-byte store per complex sample: a 2 x f64 vector, not two 8-byte halves)
#if OFS_MP_ST16
            if (a.out && st_ok) __builtin_nontemporal_store(mp_d2v{r.x, r.y}, reinterpret_cast<mp_d2v*>(&a.out[oi]));
#else
            if (a.out && st_ok) { __builtin_nontemporal_store(r.x, &a.out[oi].x); __builtin_nontemporal_store(r.y, &a.out[oi].y); }
#endif
            if (a.mag && st_ok) __builtin_nontemporal_store(mp_cabs(r), &a.mag[oi]);
#else
            if (a.out && st_ok) a.out[oi] = r;
            if (a.mag && st_ok) a.mag[oi] = mp_cabs(r);
#endif
        }
        MP_T_MARK(7);
    }
#if OFS_MP_TIMING
    if (lane == 0)
        for (int i = 0; i < 8; ++i) atomicAdd(&mp_prof[i], tacc[i]);
#endif
#undef MP_T_MARK
}

// Hbr[i] = H[bitrev(i)] / M, for the fused path; then the kernel's two 64-entry twiddle tables
// Hbr[M + l] = w^l, Hbr[M + 64 + h] = w^{64h} (from sincospi of exact ratios, once per plan)
__global__ void mc_prep_kernel(const double2* H, double2* Hbr, int M, int lb) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M + 128; i += gridDim.x * blockDim.x) {
        if (i >= M) {
            const int l = i - M;
            double sn, cs;
            sincospi(-2.0 * (double)(l < 64 ? l : 64 * (l - 64)) / (double)M, &sn, &cs);
            Hbr[i] = make_double2(cs, sn);
            continue;
        }
        const int r = (int)(__brev((unsigned)i) >> (32 - lb));
        const double2 h = H[r];
        Hbr[i] = make_double2(h.x / (double)M, h.y / (double)M);
    }
}

bool mc_fused_enabled() {                       // variant MC_FUSED=0: the rocFFT pipeline (A/B)
    return !ofs::variant_off(ofs::V_MC_FUSED);
}
bool mc_fuse_extract() {                        // variant MC_FUSE_X=0: scratch + extract kernel (A/B)
    return !ofs::variant_off(ofs::V_MC_FUSE_X);
}

// inclusive block scan of per-thread sums (fp64), returns the exclusive prefix of this thread
__device__ double block_excl_scan(double v, double* red) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    double s = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(s, d, 64);
        if (lane >= d) s += o;
    }
    if (lane == 63) red[w] = s;
    __syncthreads();
    double base = 0.0;
    for (int j = 0; j < w; ++j) base += red[j];
    __syncthreads();
    return base + s - v;
}

// one workgroup per (stream, block): outputs n = q·S + s, s in [0, S) ∩ [0, nout - q·S).
// LDS: per branch the exclusive prefix of |u_q|^2 over the block, [M + FW + 1] fp64 with one
// pad word per `per` = M / FW elements (thread t scans the contiguous chunk [t·per, (t+1)·per),
// padded so the chunk starts fall on different banks); x is read once, coalesced.
__device__ __forceinline__ int pidx(int m, int per) { return m + m / per; }

template <int FMT>
__global__ __launch_bounds__(FX) void mc_extract_kernel(McArgs a) {
    extern __shared__ double pf[];
    const int per = a.M / FX;                       // M is a power of two >= FX
    const int plen = a.M + FX + 1;                  // padded prefix length per branch (M / per = FX pads)
    double* red = pf + (size_t)a.nb * plen;
    const int64_t b = blockIdx.y, q = blockIdx.x;
    const int64_t n0 = q * a.S;
    const int ns = (int)min((int64_t)a.S, a.nout - n0);
    const int64_t g0 = n0 - (a.N - 1);
    for (int br = 0; br < a.nb; ++br) {
        const int64_t row = b * a.nb + br;
        double* P = pf + (size_t)br * plen;
        for (int m = threadIdx.x; m < a.M; m += FX) {            // |x|^2, coalesced
            const int64_t g = g0 + m;
            double e = 0.0;
            if (g >= 0 && g < a.T) { const double2 v = ldx<FMT>(a.x, row * a.T + g); e = v.x * v.x + v.y * v.y; }
            P[pidx(m, per)] = e;
        }
        __syncthreads();
        const int c0 = threadIdx.x * per;
        double loc = 0.0;
        for (int j = 0; j < per; ++j) loc += P[pidx(c0 + j, per)];
        double run = block_excl_scan(loc, red);
        for (int j = 0; j < per; ++j) {
            const int i = pidx(c0 + j, per);
            const double e = P[i];
            P[i] = run;
            run += e;
        }
        if (threadIdx.x == FX - 1) P[pidx(a.M, per)] = run;
        __syncthreads();
    }
    for (int s = threadIdx.x; s < ns; s += FX) {
        double sr = 0.0, si = 0.0, se = 0.0;
        for (int br = 0; br < a.nb; ++br) {
            const int64_t row = b * a.nb + br;
            const double2 c = a.U[(row * a.nblk + q) * a.M + (a.N - 1) + s];
            const double* P = pf + (size_t)br * plen;
            const double e = P[pidx(s + a.N, per)] - P[pidx(s, per)];   // Σ |x|^2 over the N-sample window
            if (a.mode == OFS_ZC_RAW) {
                const int64_t o = row * a.nout + n0 + s;
                if (a.out) a.out[o] = c;
                if (a.mag) a.mag[o] = hypot(c.x, c.y);
                continue;
            }
            if (a.mode == OFS_ZC_V2) {                       // zc_v2.py:493-500 combine
                const double d = a.ref_norm * sqrt(e > 1e-12 ? e : 1e-12);
                sr += c.x / d; si += c.y / d;
            } else {
                sr += c.x; si += c.y; se += e;
            }
        }
        if (a.mode == OFS_ZC_RAW) continue;
        if (a.mode == OFS_ZC_COMBINED) {                     // zc.py:113-126
            const double d = a.ref_norm * sqrt((se > 0.0 ? se : 0.0) + 1e-12);
            sr /= d; si /= d;
        }
        const int64_t o = b * a.nout + n0 + s;
        if (a.out) a.out[o] = make_double2(sr, si);
        if (a.mag) a.mag[o] = hypot(sr, si);
    }
}

size_t extract_lds(int nb, int M) { return ((size_t)nb * (M + FX + 1) + FX / 64) * sizeof(double); }

int pick_m(int N, int64_t T, int nb) {
    // overlap-save FFT size: power of two >= 2N minimising the transformed elements nblk·M
    // (ties: the smaller M), with every branch's energy prefix of a block in LDS
    const int64_t nout = T + N - 1;
    int best = 0;
    int64_t cost = INT64_MAX;
    for (int64_t M = 1; M <= (int64_t)1 << 16; M <<= 1) {
        if (M < 2 * (int64_t)N || M < FW || M < FX || extract_lds(nb, (int)M) > 160 * 1024) continue;
        const int64_t S = M - N + 1, nblk = (nout + S - 1) / S;
        if (nblk * M < cost) { cost = nblk * M; best = (int)M; }
    }
    return best;
}

rocfft_status make_plan(rocfft_plan* p, rocfft_transform_type dir, int M, int64_t batch) {
    const size_t len = (size_t)M;
    return rocfft_plan_create(p, rocfft_placement_inplace, dir, rocfft_precision_double, 1, &len, (size_t)batch,
                              nullptr);
}

}  // namespace

extern "C" {

int32_t ofs_zc_mf_plan_create(const void* ref, int32_t N, int64_t B, int32_t n_br, int64_t T, int32_t M,
                              void** plan_out, size_t* work_bytes, size_t* scratch_bytes) {
    if (!ref || !plan_out || N < 1 || B < 1 || n_br < 1 || T < 1 || M < 0 || (M && (M & (M - 1))) ||
        (M && (M < 2 * N || M < FW || M < FX)))
        return OFS_EINVAL;
    *plan_out = nullptr;
    if (!M) M = pick_m(N, T, n_br);
    if (!M || extract_lds(n_br, M) > 160 * 1024) return OFS_ETOOLONG;
    std::call_once(g_setup, [] { rocfft_setup(); });
    McPlan* p = new McPlan;
    p->N = N; p->M = M; p->S = M - N + 1; p->nb = n_br; p->B = B; p->T = T;
    p->nout = T + N - 1;
    p->nblk = (p->nout + p->S - 1) / p->S;
    const int64_t batch = B * n_br * p->nblk;
    p->scratch_bytes = (size_t)batch * M * sizeof(double2);
    rocfft_status s = make_plan(&p->fwd, rocfft_transform_type_complex_forward, M, batch);
    if (s == rocfft_status_success) s = make_plan(&p->inv, rocfft_transform_type_complex_inverse, M, batch);
    size_t w1 = 0, w2 = 0;
    if (s == rocfft_status_success) s = rocfft_plan_get_work_buffer_size(p->fwd, &w1);
    if (s == rocfft_status_success) s = rocfft_plan_get_work_buffer_size(p->inv, &w2);
    p->work_bytes = w1 > w2 ? w1 : w2;
    // H = FFT_M(h), h[i] = conj(ref[N-1-i]) (host build, one batch-1 transform on the device)
    double2* hh = nullptr;
    rocfft_plan p1 = nullptr;
    bool ok = s == rocfft_status_success && hipMalloc(&p->H, (size_t)M * sizeof(double2)) == hipSuccess &&
              hipHostMalloc(&hh, (size_t)M * sizeof(double2)) == hipSuccess;
    if (ok) {
        const double2* r = static_cast<const double2*>(ref);
        double nrm = 0.0;
        for (int i = 0; i < M; ++i) hh[i] = make_double2(0.0, 0.0);
        for (int i = 0; i < N; ++i) {
            const double2 v = r[N - 1 - i];
            hh[i] = make_double2(v.x, -v.y);
            nrm += v.x * v.x + v.y * v.y;
        }
        p->ref_norm = sqrt(nrm);
        ok = hipMemcpy(p->H, hh, (size_t)M * sizeof(double2), hipMemcpyHostToDevice) == hipSuccess &&
             make_plan(&p1, rocfft_transform_type_complex_forward, M, 1) == rocfft_status_success;
    }
    if (ok) {
        size_t w = 0;
        void* wk = nullptr;
        rocfft_execution_info info = nullptr;
        ok = rocfft_plan_get_work_buffer_size(p1, &w) == rocfft_status_success &&
             (w == 0 || hipMalloc(&wk, w) == hipSuccess) &&
             rocfft_execution_info_create(&info) == rocfft_status_success &&
             (w == 0 || rocfft_execution_info_set_work_buffer(info, wk, w) == rocfft_status_success);
        void* io[1] = {p->H};
        if (ok) ok = rocfft_execute(p1, io, nullptr, info) == rocfft_status_success && hipDeviceSynchronize() == hipSuccess;
        if (info) rocfft_execution_info_destroy(info);
        if (wk) (void)hipFree(wk);
    }
    if (p1) rocfft_plan_destroy(p1);
    if (hh) (void)hipHostFree(hh);
    if (!ok) {
        if (p->fwd) rocfft_plan_destroy(p->fwd);
        if (p->inv) rocfft_plan_destroy(p->inv);
        if (p->H) (void)hipFree(p->H);
        delete p;
        return OFS_EFFT;
    }
    // per-plan, once: the execution info and the extract kernels' LDS limit (per call they cost
    // host time comparable to the whole GPU pipeline at this size)
    const size_t lds = extract_lds(p->nb, p->M);
    bool ok2 = rocfft_execution_info_create(&p->info) == rocfft_status_success;
    if (ok2 && p->M == MF_M) {                  // fused path resources (optional: rocFFT otherwise)
        if (hipMalloc(&p->Hbr, (size_t)(MF_M + 128) * sizeof(double2)) == hipSuccess) {
            hipLaunchKernelGGL(mc_prep_kernel, dim3(MF_M / 256 + 1), dim3(256), 0, 0, p->H, p->Hbr, MF_M, 13);
            const size_t fl = MF_LDS;
            const bool okf = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
                hipFuncSetAttribute((const void*)mc_fused_kernel<OFS_C64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fl) == hipSuccess &&
                hipFuncSetAttribute((const void*)mc_fused_kernel<OFS_C128, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fl) == hipSuccess &&
                hipFuncSetAttribute((const void*)mc_fused_kernel<OFS_CI16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fl) == hipSuccess &&
                hipFuncSetAttribute((const void*)mc_fused_kernel<OFS_C64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fl) == hipSuccess &&
                hipFuncSetAttribute((const void*)mc_fused_kernel<OFS_C128, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fl) == hipSuccess &&
                hipFuncSetAttribute((const void*)mc_fused_kernel<OFS_CI16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fl) == hipSuccess;
            if (!okf) {
                (void)hipFree(p->Hbr);
                p->Hbr = nullptr;
            } else {
                int dev = 0, ncu = 0;
                const int pl = MP_LDS;
                if (hipGetDevice(&dev) == hipSuccess &&
                    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                    hipFuncSetAttribute((const void*)mc_pers_kernel<OFS_C64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, pl) == hipSuccess &&
                    hipFuncSetAttribute((const void*)mc_pers_kernel<OFS_C128, false>, hipFuncAttributeMaxDynamicSharedMemorySize, pl) == hipSuccess &&
                    hipFuncSetAttribute((const void*)mc_pers_kernel<OFS_CI16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, pl) == hipSuccess &&
                    hipFuncSetAttribute((const void*)mc_pers_kernel<OFS_C64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, pl) == hipSuccess &&
                    hipFuncSetAttribute((const void*)mc_pers_kernel<OFS_C128, true>, hipFuncAttributeMaxDynamicSharedMemorySize, pl) == hipSuccess &&
                    hipFuncSetAttribute((const void*)mc_pers_kernel<OFS_CI16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, pl) == hipSuccess)
                    p->n_cu = ncu > 0 ? ncu : 0;
            }
        } else {
            p->Hbr = nullptr;
        }
    }
    if (!ok2) {
        if (p->info) rocfft_execution_info_destroy(p->info);
        rocfft_plan_destroy(p->fwd);
        rocfft_plan_destroy(p->inv);
        (void)hipFree(p->H);
        delete p;
        return OFS_EHIP;
    }
    if (work_bytes) *work_bytes = p->work_bytes;
    if (scratch_bytes) *scratch_bytes = p->scratch_bytes;
    *plan_out = p;
    return OFS_OK;
}

int32_t ofs_zc_mf_plan_destroy(void* plan) {
    McPlan* p = static_cast<McPlan*>(plan);
    if (!p) return OFS_OK;
    if (p->info) rocfft_execution_info_destroy(p->info);
    if (p->fwd) rocfft_plan_destroy(p->fwd);
    if (p->inv) rocfft_plan_destroy(p->inv);
    if (p->H) (void)hipFree(p->H);
    if (p->Hbr) (void)hipFree(p->Hbr);
    delete p;
    return OFS_OK;
}

int32_t ofs_zc_correlate_fft(void* plan, int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                             double ref_energy, int32_t mode, void* corr, double* corr_mag, void* scratch,
                             void* work, void* stream) {
    McPlan* p = static_cast<McPlan*>(plan);
    if (!p || !x || !scratch || (in_fmt != OFS_C64 && in_fmt != OFS_C128 && in_fmt != OFS_CI16) ||
        B != p->B || n_br != p->nb || T != p->T || (!corr && !corr_mag) ||
        (mode != OFS_ZC_RAW && mode != OFS_ZC_V2 && mode != OFS_ZC_COMBINED && mode != OFS_ZC_SUM) ||
        (p->work_bytes && !work) || !(ref_energy >= 0.0))
        return OFS_EINVAL;
    hipStream_t st = static_cast<hipStream_t>(stream);
    McArgs a{x, T, n_br, p->N, p->M, p->S, p->nblk, p->nout, mode, sqrt(ref_energy), static_cast<double2*>(scratch),
             p->H, static_cast<double2*>(corr), corr_mag};
    const int64_t rows = B * n_br;
    if (p->Hbr && mc_fused_enabled() && rows * p->nblk <= 0x7fffffff) {
        const dim3 gf((unsigned)(rows * p->nblk));
        const size_t fl = MF_LDS;
        const bool fx = n_br == 1 && mc_fuse_extract();             // one branch: no scratch round trip
        const int64_t total = rows * p->nblk;
        const bool pers = p->n_cu > 0 && !ofs::variant_off(ofs::V_MC_PERS);
        const dim3 gpers((unsigned)std::min<int64_t>(total, p->n_cu));
        const size_t pl = MP_LDS;
#define MF_GO(F)                                                                                      \
        if (pers && fx) hipLaunchKernelGGL((mc_pers_kernel<F, true>), gpers, dim3(MP_T), pl, st, a, p->Hbr, total); \
        else if (pers) hipLaunchKernelGGL((mc_pers_kernel<F, false>), gpers, dim3(MP_T), pl, st, a, p->Hbr, total); \
        else if (fx) hipLaunchKernelGGL((mc_fused_kernel<F, true>), gf, dim3(MF_T), fl, st, a, p->Hbr);     \
        else hipLaunchKernelGGL((mc_fused_kernel<F, false>), gf, dim3(MF_T), fl, st, a, p->Hbr);
        switch (in_fmt) {
            case OFS_C64: MF_GO(OFS_C64) break;
            case OFS_C128: MF_GO(OFS_C128) break;
            default: MF_GO(OFS_CI16) break;
        }
#undef MF_GO
        if (hipGetLastError() != hipSuccess) return OFS_EHIP;
        if (fx) return OFS_OK;
        const size_t lds = extract_lds(n_br, p->M);
        const dim3 ge((unsigned)p->nblk, (unsigned)B);
        switch (in_fmt) {
            case OFS_C64: hipLaunchKernelGGL(mc_extract_kernel<OFS_C64>, ge, dim3(FX), lds, st, a); break;
            case OFS_C128: hipLaunchKernelGGL(mc_extract_kernel<OFS_C128>, ge, dim3(FX), lds, st, a); break;
            default: hipLaunchKernelGGL(mc_extract_kernel<OFS_CI16>, ge, dim3(FX), lds, st, a); break;
        }
        return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
    }
    const dim3 gp((unsigned)((p->M + FW - 1) / FW), (unsigned)(rows * p->nblk));
    switch (in_fmt) {
        case OFS_C64: hipLaunchKernelGGL(mc_pack_kernel<OFS_C64>, gp, dim3(FW), 0, st, a); break;
        case OFS_C128: hipLaunchKernelGGL(mc_pack_kernel<OFS_C128>, gp, dim3(FW), 0, st, a); break;
        default: hipLaunchKernelGGL(mc_pack_kernel<OFS_CI16>, gp, dim3(FW), 0, st, a); break;
    }
    if (hipGetLastError() != hipSuccess) return OFS_EHIP;
    rocfft_execution_info info = p->info;
    rocfft_status s = rocfft_execution_info_set_stream(info, st);
    if (s == rocfft_status_success && p->work_bytes) s = rocfft_execution_info_set_work_buffer(info, work, p->work_bytes);
    void* io[1] = {scratch};
    if (s == rocfft_status_success) s = rocfft_execute(p->fwd, io, nullptr, info);
    if (s == rocfft_status_success) {
        const int64_t n = rows * p->nblk * p->M;
        hipLaunchKernelGGL(mc_mul_kernel, dim3((unsigned)std::min<int64_t>((n + FW - 1) / FW, 1 << 20)), dim3(FW), 0, st,
                           static_cast<double2*>(scratch), p->H, n, p->M, 1.0 / (double)p->M);
        if (hipGetLastError() != hipSuccess) return OFS_EHIP;
        s = rocfft_execute(p->inv, io, nullptr, info);
    }
    if (s != rocfft_status_success) return OFS_EFFT;
    const size_t lds = extract_lds(n_br, p->M);      // its LDS limit was raised at plan creation
    const dim3 ge((unsigned)p->nblk, (unsigned)B);
    switch (in_fmt) {
        case OFS_C64: hipLaunchKernelGGL(mc_extract_kernel<OFS_C64>, ge, dim3(FX), lds, st, a); break;
        case OFS_C128: hipLaunchKernelGGL(mc_extract_kernel<OFS_C128>, ge, dim3(FX), lds, st, a); break;
        default: hipLaunchKernelGGL(mc_extract_kernel<OFS_CI16>, ge, dim3(FX), lds, st, a); break;
    }
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

#if OFS_MP_TIMING
// per-phase cycle totals of mc_pers_kernel (summed over waves) since the last call (diagnostic builds)
int32_t ofs_mp_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mp_prof), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(mp_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
}  // extern "C"
