// win_fast.hip — streaming fast path of the sliding-window timing metrics, fp32, any T:
//   S&C            sc.sc_streaming_metric                       (sc.py:42-78)
//   combined S&C   combined_sc_min.schmidl_cox_streaming_metric (combined_sc_min.py:116-164)
//   Minn           minn.minn_streaming_metric(_parameterized)   (minn.py:59-112, :697-751)
//
// All three are window sums of one lagged product and of the energy, read at a few lags,
// written in trailing form around the newest sample n = d + N - 1 (output index d):
//   a(j) = x[j]·conj(x[j-D]),  S_a(n) = Σ_{j=n-W+1..n} a(j),  S_e(n) = Σ |x[j]|² (same window)
//   S&C      (D = W = N/2):  P = conj(S_a(n)),  R = S_e(n)
//   combined (D = W = N/2):  P = conj(S_a(n)),  R = S_e(n) + S_e(n-W)
//   Minn     (D = W = N/4):  P = conj(S_a(n) + S_a(n-2W)),  R = S_e(n) + S_e(n-W) + S_e(n-2W)
// (q0·conj(q1) = conj(a) over the window ending at d+2Q-1, etc.)
//
// Layout is the one of aa_fast.hip: one wave per stream, rows of RL = 64·E samples, lane l
// owns samples RL·k + E·l + e, and with W = MW·RL every lag (D, W, 2W) lands in the SAME lane
// and element MW or 2MW rows back — the lagged sample, the retained window suffix and the
// window sums at n-W / n-2W live in register rings indexed by k mod (ring), resolved at
// compile time by unrolling the row loop by the ring period.  Window sums use the
// cancellation-free split S = suffix(row k-MW) + rows between (fp64 row totals) + prefix(row
// k) of aa_fast.  Rows stream from HBM into registers one row ahead (software pipelined),
// so the kernel handles streams of any length (cfg4: 4096 samples, N = 2048).
#include "ofs_common.h"
#include "ofdmsync.h"

using namespace ofs;

namespace {

#ifndef OFS_WF_WG
#define OFS_WF_WG 256
#endif
constexpr int WF_WG = OFS_WF_WG;       // 4 waves = 4 streams per workgroup (tuning builds: 64)
enum { WF_SC = 1, WF_COMB = 2, WF_MINN = 3 };
typedef float wf4u __attribute__((ext_vector_type(4), aligned(8)));   // pair loads / stores at 8-byte alignment
typedef float wf2u __attribute__((ext_vector_type(2), aligned(4)));
typedef float wf4ua __attribute__((ext_vector_type(4), aligned(4)));

// packed fp32 pairs (re, im): products, partials and window sums issue as v_pk_* (see the fused
// kernel below); conj(c)·d accumulated, so P = Σ conj(a) needs no negation
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 cjmul_acc(pf2 c, pf2 d, pf2 acc) {
    acc = __builtin_elementwise_fma(c.xx, d, acc);
    return __builtin_elementwise_fma(c.yy, pf2{d.y, -d.x}, acc);
}

template <int MODE, int E, int MW, int NB>
__global__ __launch_bounds__(WF_WG) void win_fast_kernel(WinFastArgs a) {
    constexpr int RL = 64 * E;
    constexpr int W = MW * RL;
    constexpr int N = (MODE == WF_MINN) ? 4 * W : 2 * W;
    constexpr int HR = (MODE == WF_MINN) ? 2 * MW : MW;     // history ring rows (COMB / MINN)
    constexpr int PD = 2;                                    // rows in flight ahead of use
    constexpr int PER = HR > PD ? HR : PD;                   // unroll period (ring sizes divide it)
    constexpr int V4 = E / 2;                                // float4 loads per lane per row
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)xcd_block_w() * (WF_WG / 64) + (threadIdx.x >> 6);
    if (b >= a.B) return;
    const int64_t T = a.T;
    const int64_t nout = T - N + 1;
    const int nrows = (int)((T + RL - 1) / RL);
    const float2* xb = reinterpret_cast<const float2*>(a.x) + b * NB * T;   // [NB][T] of stream b
    float* Mo = a.M ? reinterpret_cast<float*>(a.M) + b * nout : nullptr;
    float2* Po = a.P ? reinterpret_cast<float2*>(a.P) + b * nout : nullptr;
    float* Ro = a.R ? reinterpret_cast<float*>(a.R) + b * nout : nullptr;

    pf2 lx[NB][MW][E];                           // x of rows k-MW..k-1 (lag D = W), per branch
    pf2 sS[MW][E];                               // retained in-window suffixes (conj products)
    float sE[MW][E];
    pf2 hS[HR][E];                               // window sums of past rows (MINN: products)
    float hE[HR][E];                             // (COMB / MINN: energies)
    double cbR[MW], cbI[MW], cbE[MW];            // row bases C[j] for j in (k-MW, k]
    double CR = 0.0, CI = 0.0, CE = 0.0;         // C[k]: prefix at the start of row k
#pragma unroll
    for (int m = 0; m < MW; ++m) {
        cbR[m] = 0.0; cbI[m] = 0.0; cbE[m] = 0.0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            sS[m][e] = pf2{0.f, 0.f}; sE[m][e] = 0.f;
#pragma unroll
            for (int t = 0; t < NB; ++t) lx[t][m][e] = pf2{0.f, 0.f};
        }
    }
#pragma unroll
    for (int m = 0; m < HR; ++m)
#pragma unroll
        for (int e = 0; e < E; ++e) { hS[m][e] = pf2{0.f, 0.f}; hE[m][e] = 0.f; }

    float4 nx[PD][NB][V4];
    // whole rows: 8-byte-aligned float4 pair loads (any T: stream bases are float2-aligned);
    // the last, partial row per sample with zeros past T (wave-uniform choice)
    auto load_row = [&](int k, float4 (&dst)[NB][V4]) {
        const int64_t n0 = (int64_t)RL * k + E * lane;
        const bool whole = (int64_t)RL * (k + 1) <= T;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const float2* xs = xb + (int64_t)t * T;
#pragma unroll
            for (int j = 0; j < V4; ++j) {
                if (whole) {
                    const wf4u v = *reinterpret_cast<const wf4u*>(xs + n0 + 2 * j);
                    dst[t][j] = make_float4(v.x, v.y, v.z, v.w);
                } else {
                    const int64_t m0 = n0 + 2 * j;
                    const float2 u0 = m0 < T ? xs[m0] : make_float2(0.f, 0.f);
                    const float2 u1 = m0 + 1 < T ? xs[m0 + 1] : make_float2(0.f, 0.f);
                    dst[t][j] = make_float4(u0.x, u0.y, u1.x, u1.y);
                }
            }
        }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) load_row(p < nrows ? p : 0, nx[p]);

    for (int k0 = 0; k0 < nrows; k0 += PER) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = k0 + u;
            if (k < nrows) {
                const int sl = u % MW;                              // ring slot of row k (and k-MW)
                // ---- lagged products conj(x[j])·x[j-D] and energies, summed over the branches ----
                pf2 av[E];
                float aE[E];
#pragma unroll
                for (int e = 0; e < E; ++e) { av[e] = pf2{0.f, 0.f}; aE[e] = 0.f; }
#pragma unroll
                for (int t = 0; t < NB; ++t) {
#pragma unroll
                    for (int e = 0; e < E; ++e) {                   // zeros past T from load_row
                        const float4 v = nx[u % PD][t][e / 2];
                        const pf2 c = (e & 1) ? pf2{v.z, v.w} : pf2{v.x, v.y};
                        aE[e] += fmaf(c.x, c.x, c.y * c.y);
                        if (k >= MW) av[e] = cjmul_acc(c, lx[t][sl][e], av[e]);
                        lx[t][sl][e] = c;
                    }
                }
                if (k + PD < nrows) load_row(k + PD, nx[u % PD]);   // PD rows ahead
                // ---- in-lane partials (forward f, backward g) ----
                pf2 fS[E], gS[E];
                float fE[E], gE[E];
                fS[0] = av[0]; fE[0] = aE[0];
#pragma unroll
                for (int e = 1; e < E; ++e) { fS[e] = fS[e - 1] + av[e]; fE[e] = fE[e - 1] + aE[e]; }
                gS[E - 1] = pf2{0.f, 0.f}; gE[E - 1] = 0.f;
#pragma unroll
                for (int e = E - 2; e >= 0; --e) { gS[e] = gS[e + 1] + av[e + 1]; gE[e] = gE[e + 1] + aE[e + 1]; }
                // ---- lane totals: fp64 wave scan; row totals; rows strictly inside the window ----
                const double iR = scan_add((double)fS[E - 1].x), iI = scan_add((double)fS[E - 1].y), iE = scan_add((double)fE[E - 1]);
                const double tR = readlane(iR, 63), tI = readlane(iI, 63), tE = readlane(iE, 63);
                const pf2 xS = pf2{(float)shr1z(iR), (float)shr1z(iI)}, uS = pf2{(float)(tR - iR), (float)(tI - iI)};
                const float xE = (float)shr1z(iE), uE = (float)(tE - iE);
                const int so = (u + 1) % MW;                        // slot of C[k-MW+1]
                const pf2 wS = k >= MW ? pf2{(float)(CR - cbR[so]), (float)(CI - cbI[so])} : pf2{(float)CR, (float)CI};
                const float wE = (float)(k >= MW ? CE - cbE[so] : CE);
                // ---- window sums, outputs ----
                float oM[E], oR[E];
                pf2 oP[E];
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    pf2 S = wS + (xS + fS[e]);
                    float SE = wE + (xE + fE[e]);
                    if (k >= MW) { S += sS[sl][e]; SE += sE[sl][e]; }
                    sS[sl][e] = uS + gS[e]; sE[sl][e] = uE + gE[e];
                    pf2 P = S;
                    float RR = SE;
                    if constexpr (MODE == WF_COMB) {
                        RR += hE[sl][e];                            // S_e(n - W): row k-MW
                        hE[sl][e] = SE;
                    } else if constexpr (MODE == WF_MINN) {
                        const int h2 = u % HR;                      // row k-2MW (and k)
                        const int h1 = (u + MW) % HR;               // row k-MW
                        P += hS[h2][e];
                        RR += hE[h1][e] + hE[h2][e];
                        hS[h2][e] = S; hE[h2][e] = SE;
                    }
                    const float den = fmaxf(RR, 1e-12f);
                    const float num = (MODE == WF_MINN) ? fmaxf(P.x, 0.f) * fmaxf(P.x, 0.f) : fmaf(P.x, P.x, P.y * P.y);
                    oM[e] = num * __builtin_amdgcn_rcpf(den * den);
                    oP[e] = P; oR[e] = RR;
                }
                // C[k+1] replaces C[k-MW+1] in the ring
                cbR[so] = CR + tR; cbI[so] = CI + tI; cbE[so] = CE + tE;
                CR += tR; CI += tI; CE += tE;
                // ---- stores: outputs d = n - (N-1) in [0, nout) ----
                // a lane's E outputs are contiguous: dword-aligned vector stores (the output
                // rows [B][T-N+1] are not 16-byte aligned; gfx950 global stores allow it)
                const int64_t d0 = (int64_t)RL * k + E * lane - (N - 1);
                if (d0 >= 0 && d0 + E <= nout) {
                    if constexpr (E >= 4) {
#pragma unroll
                        for (int j = 0; j < E; j += 4) {
                            if (Mo) *reinterpret_cast<wf4ua*>(Mo + d0 + j) = wf4ua{oM[j], oM[j + 1], oM[j + 2], oM[j + 3]};
                            if (Ro) *reinterpret_cast<wf4ua*>(Ro + d0 + j) = wf4ua{oR[j], oR[j + 1], oR[j + 2], oR[j + 3]};
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < E; j += 2) {
                            if (Mo) *reinterpret_cast<wf2u*>(Mo + d0 + j) = wf2u{oM[j], oM[j + 1]};
                            if (Ro) *reinterpret_cast<wf2u*>(Ro + d0 + j) = wf2u{oR[j], oR[j + 1]};
                        }
                    }
#pragma unroll
                    for (int j = 0; j < E; j += 2)
                        if (Po) *reinterpret_cast<wf4u*>(Po + d0 + j) = wf4u{oP[j].x, oP[j].y, oP[j + 1].x, oP[j + 1].y};
                } else {
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int64_t d = d0 + e;
                        if (d >= 0 && d < nout) {
                            if (Mo) Mo[d] = oM[e];
                            if (Po) Po[d] = make_float2(oP[e].x, oP[e].y);
                            if (Ro) Ro[d] = oR[e];
                        }
                    }
                }
            }
        }
    }
}

// Realigned row stores (OFS_SCM_ALIGN == 2): a lane owns 4 consecutive outputs at rowp + 4·lane,
// which for 3 of 4 output rows [B][T-N+1] is not a 16-byte boundary.  Each lane instead stores the
// aligned 16-byte chunk that ends inside its group, taking the leading o values from lane - 1
// (DPP wave_shr:1); lane 0 stores its own leading 4 - o values and lane 63 its trailing o values
// (the chunks straddling the neighbour rows).  o is wave-uniform.
__device__ __forceinline__ float shr1f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
typedef float wf3u __attribute__((ext_vector_type(3), aligned(4)));
__device__ __forceinline__ void store_al4(float* rowp, const float (&v)[4], int lane) {
    const int o = (int)(((uintptr_t)rowp >> 2) & 3);
    float* p = rowp + 4 * lane;
    const float p1 = shr1f(v[1]), p2 = shr1f(v[2]), p3 = shr1f(v[3]);
    if (o == 0) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else if (o == 1) {
        if (lane) *reinterpret_cast<float4*>(p - 1) = make_float4(p3, v[0], v[1], v[2]);
        else *reinterpret_cast<wf3u*>(p) = wf3u{v[0], v[1], v[2]};
        if (lane == 63) p[3] = v[3];
    } else if (o == 2) {
        if (lane) *reinterpret_cast<float4*>(p - 2) = make_float4(p2, p3, v[0], v[1]);
        else *reinterpret_cast<wf2u*>(p) = wf2u{v[0], v[1]};
        if (lane == 63) *reinterpret_cast<wf2u*>(p + 2) = wf2u{v[2], v[3]};
    } else {
        if (lane) *reinterpret_cast<float4*>(p - 3) = make_float4(p1, p2, p3, v[0]);
        else p[0] = v[0];
        if (lane == 63) *reinterpret_cast<wf3u*>(p + 1) = wf3u{v[1], v[2], v[3]};
    }
}
// complex outputs: 16 bytes = 2 values, so the group is 8-byte-shifted or aligned
__device__ __forceinline__ void store_al2(float2* rowp, const float (&re)[4], const float (&im)[4], int lane) {
    float2* p = rowp + 4 * lane;
    const float qr = shr1f(re[3]), qi = shr1f(im[3]);
    if ((((uintptr_t)rowp >> 3) & 1) == 0) {
        *reinterpret_cast<float4*>(p) = make_float4(re[0], im[0], re[1], im[1]);
        *reinterpret_cast<float4*>(p + 2) = make_float4(re[2], im[2], re[3], im[3]);
    } else {
        if (lane) *reinterpret_cast<float4*>(p - 1) = make_float4(qr, qi, re[0], im[0]);
        else p[0] = make_float2(re[0], im[0]);
        *reinterpret_cast<float4*>(p + 1) = make_float4(re[1], im[1], re[2], im[2]);
        if (lane == 63) p[3] = make_float2(re[3], im[3]);
    }
}

// ------------------------------------------------------------------------------------------
// Fused combined_sc_min detector (cfg4): combined S&C (D = W = 2Q, R over both halves) AND
// Minn (D = W = Q) from ONE pass over the stream, N = 4Q.  Lags in rows: Q = MW rows.
//   S&C : P = conj(S_h(n)),            R = S_e(n) + S_e(n-Q) + S_e(n-2Q) + S_e(n-3Q)
//   Minn: P = conj(S_q(n) + S_q(n-2Q)), R = S_e(n) + S_e(n-Q) + S_e(n-2Q)
// with S_h / S_q the lag-2Q / lag-Q product windows and S_e the Q-window energy.  The x ring
// (2MW rows) and the window suffixes stay in registers; the per-row histories of S_e and S_q
// (read back Q..3Q later) live in a per-wave LDS slice (no barriers: one wave owns it).
// ------------------------------------------------------------------------------------------
struct WinFusedArgs {
    const void* x; int64_t B, T; int N;
    float* Ms; float2* Ps; float* Rs; float* Mm; float2* Pm; float* Rm;
};

// 16-byte-aligned output rows of the fused kernel (row origin shift).  Paired A/B (tools/lib_ab.py
// --op scminn, r02r): 0.720 vs 0.711 ms on the cfg4 shard, 0.618 vs 0.576 ms with two branches -
// slower than the misaligned 8-byte stores despite the flat SOL probe's 0.70 vs 0.60, so off.
#ifndef OFS_SCM_ALIGN
#define OFS_SCM_ALIGN 0
#endif
// occupancy bound (min waves per SIMD) of the fused kernel; tuning builds set -DOFS_SCM_WAVES=N
#ifndef OFS_SCM_WAVES
#define OFS_SCM_WAVES 0
#endif
// workgroup size of the fused kernels by branch count: two branches run 2 waves (streams) per
// workgroup - paired (round 6, tools/libs_cfg_ab.sh, profiles/r06t_cfg4_workgroup_ab.txt): cfg4_2br
// 0.4367 ms at 4 waves, 0.4159 at 2, 0.4225 at 1; one branch (cfg4) keeps 4 (5.30 vs 5.50 / 5.74 ms)
#ifndef OFS_SCM_WG2
#define OFS_SCM_WG2 128
#endif
constexpr int scm_wg(int nb) { return nb == 2 ? OFS_SCM_WG2 : WF_WG; }
#if OFS_SCM_WAVES > 0
#define OFS_SCM_BOUNDS __launch_bounds__(scm_wg(NB), OFS_SCM_WAVES)
#else
#define OFS_SCM_BOUNDS __launch_bounds__(scm_wg(NB))
#endif

template <int E, int MW, int NB>
__global__ OFS_SCM_BOUNDS void sc_minn_fast_kernel(WinFusedArgs a) {
    constexpr int RL = 64 * E;
    constexpr int N = 4 * MW * RL;
    constexpr int XR = 2 * MW;                  // x ring / S_h suffix ring / S_q history ring
    constexpr int ER = 4 * MW;                  // S_e history ring
    constexpr int PD = 2;
    constexpr int PER = ER;
    constexpr int V4 = E / 2;
    constexpr int WG = scm_wg(NB);
    __shared__ float hist[WG / 64][ER + 2 * XR][E][64];   // [S_e rows | S_q re rows | S_q im rows]
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t b = (int64_t)xcd_block_w() * (WG / 64) + w;
    if (b >= a.B) return;
    const int64_t T = a.T;
    const int64_t nout = T - N + 1;
    // Row origin shift (OFS_SCM_ALIGN): the [B][T-N+1] output rows have odd length, so a lane's E
    // outputs would start 4-byte-misaligned for 3 of 4 streams; starting the rows s samples
    // before the stream (zeros there) puts every full lane group of outputs on a 16-byte boundary
    // (flat SOL probe of this 1 : 4 read : write mix: 0.70 of peak with aligned 16-B stores
    // against 0.60 with misaligned 8-B ones).  Inputs then load 8-byte-aligned (f4u).
    const int64_t s = OFS_SCM_ALIGN == 1 ? (((b * nout - (N - 1)) % 4) + 4) % 4 : 0;
    const int nrows = (int)((T + s + RL - 1) / RL);
    const float2* xb = reinterpret_cast<const float2*>(a.x) + b * NB * T;   // [NB][T] of stream b

    float xr_[NB][XR][E], xi_[NB][XR][E];
    float shR[XR][E], shI[XR][E];               // S_h suffixes (window 2Q = XR rows)
    float sqR[MW][E], sqI[MW][E], seE[MW][E];   // S_q, S_e suffixes (window Q = MW rows)
    double chR[XR], chI[XR], cqR[MW], cqI[MW], ceE[MW];
    double CHR = 0, CHI = 0, CQR = 0, CQI = 0, CEE = 0;
#pragma unroll
    for (int m = 0; m < XR; ++m) {
        chR[m] = 0; chI[m] = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            shR[m][e] = 0.f; shI[m][e] = 0.f;
#pragma unroll
            for (int t = 0; t < NB; ++t) { xr_[t][m][e] = 0.f; xi_[t][m][e] = 0.f; }
        }
    }
#pragma unroll
    for (int m = 0; m < MW; ++m) {
        cqR[m] = 0; cqI[m] = 0; ceE[m] = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) { sqR[m][e] = 0.f; sqI[m][e] = 0.f; seE[m][e] = 0.f; }
    }
    auto H = [&](int row, int e) -> float& { return hist[w][row][e][lane]; };

    float4 nx[PD][NB][V4];
    // row k = samples [RL·k - s, RL·(k+1) - s): pairs as 8-byte-aligned float4 when the row lies
    // inside the stream, else per sample with zeros outside [0, T) (wave-uniform choice)
    auto load_row = [&](int k, float4 (&dst)[NB][V4]) {
        const int64_t r0 = (int64_t)RL * k - s;
        const int64_t n0 = r0 + E * lane;
        const bool whole = r0 >= 0 && r0 + RL <= T;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const float2* xs = xb + (int64_t)t * T;
            if (whole) {
#pragma unroll
                for (int j = 0; j < V4; ++j) {
                    const wf4u v = *reinterpret_cast<const wf4u*>(xs + n0 + 2 * j);
                    dst[t][j] = make_float4(v.x, v.y, v.z, v.w);
                }
            } else {
#pragma unroll
                for (int j = 0; j < V4; ++j) {
                    const int64_t m0 = n0 + 2 * j, m1 = m0 + 1;
                    const float2 u0 = (m0 >= 0 && m0 < T) ? xs[m0] : make_float2(0.f, 0.f);
                    const float2 u1 = (m1 >= 0 && m1 < T) ? xs[m1] : make_float2(0.f, 0.f);
                    dst[t][j] = make_float4(u0.x, u0.y, u1.x, u1.y);
                }
            }
        }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) load_row(p < nrows ? p : 0, nx[p]);

    // in-lane forward/backward partials + fp64 wave scan of one quantity
    struct Part { float f[E], g[E]; float xe, us; double tot; };
    auto part = [&](const float (&v)[E], Part& p) {
        p.f[0] = v[0];
#pragma unroll
        for (int e = 1; e < E; ++e) p.f[e] = p.f[e - 1] + v[e];
        p.g[E - 1] = 0.f;
#pragma unroll
        for (int e = E - 2; e >= 0; --e) p.g[e] = p.g[e + 1] + v[e + 1];
        const double i = scan_add((double)p.f[E - 1]);
        p.tot = readlane(i, 63);
        p.xe = (float)shr1z(i);
        p.us = (float)(p.tot - i);
    };

    for (int k0 = 0; k0 < nrows; k0 += PER) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = k0 + u;
            if (k < nrows) {
                const int64_t nb = (int64_t)RL * k + E * lane - s;
                const int x2 = u % XR;                 // row k-2MW (x ring), then row k
                const int x1 = (u + MW) % XR;          // row k-MW
                float hR[E], hI[E], qR[E], qI[E], en[E];
#pragma unroll
                for (int e = 0; e < E; ++e) { hR[e] = 0.f; hI[e] = 0.f; qR[e] = 0.f; qI[e] = 0.f; en[e] = 0.f; }
#pragma unroll
                for (int t = 0; t < NB; ++t) {         // products summed over the branches
                    float cr[E], ci[E];
#pragma unroll
                    for (int j = 0; j < V4; ++j) {     // zeros outside [0, T) come from load_row
                        const float4 v = nx[u % PD][t][j];
                        cr[2 * j] = v.x; ci[2 * j] = v.y;
                        cr[2 * j + 1] = v.z; ci[2 * j + 1] = v.w;
                    }
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        en[e] += fmaf(cr[e], cr[e], ci[e] * ci[e]);
                        const float d2r = xr_[t][x2][e], d2i = xi_[t][x2][e], d1r = xr_[t][x1][e], d1i = xi_[t][x1][e];
                        hR[e] += fmaf(cr[e], d2r, ci[e] * d2i); hI[e] += fmaf(ci[e], d2r, -(cr[e] * d2i));
                        qR[e] += fmaf(cr[e], d1r, ci[e] * d1i); qI[e] += fmaf(ci[e], d1r, -(cr[e] * d1i));
                        xr_[t][x2][e] = cr[e]; xi_[t][x2][e] = ci[e];
                    }
                }
                if (k + PD < nrows) load_row(k + PD, nx[u % PD]);
                Part ph_r, ph_i, pq_r, pq_i, pe;
                part(hR, ph_r); part(hI, ph_i); part(qR, pq_r); part(qI, pq_i); part(en, pe);
                const int sq = u % MW, soq = (u + 1) % MW, soh = (u + 1) % XR;
                const float whR = (float)(k >= XR ? CHR - chR[soh] : CHR);
                const float whI = (float)(k >= XR ? CHI - chI[soh] : CHI);
                const float wqR = (float)(k >= MW ? CQR - cqR[soq] : CQR);
                const float wqI = (float)(k >= MW ? CQI - cqI[soq] : CQI);
                const float weE = (float)(k >= MW ? CEE - ceE[soq] : CEE);
                const int e0 = u % ER, e1 = (u + 3 * MW) % ER, e2 = (u + 2 * MW) % ER, e3 = (u + MW) % ER;
                float oMs[E], oRs[E], oMm[E], oRm[E], oPsr[E], oPsi[E], oPmr[E], oPmi[E];
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    float SHR = whR + (ph_r.xe + ph_r.f[e]), SHI = whI + (ph_i.xe + ph_i.f[e]);
                    float SQR = wqR + (pq_r.xe + pq_r.f[e]), SQI = wqI + (pq_i.xe + pq_i.f[e]);
                    float SE = weE + (pe.xe + pe.f[e]);
                    if (k >= XR) { SHR += shR[x2][e]; SHI += shI[x2][e]; }
                    if (k >= MW) { SQR += sqR[sq][e]; SQI += sqI[sq][e]; SE += seE[sq][e]; }
                    shR[x2][e] = ph_r.us + ph_r.g[e]; shI[x2][e] = ph_i.us + ph_i.g[e];
                    sqR[sq][e] = pq_r.us + pq_r.g[e]; sqI[sq][e] = pq_i.us + pq_i.g[e];
                    seE[sq][e] = pe.us + pe.g[e];
                    // histories (LDS): S_e rows k-MW, k-2MW, k-3MW; S_q row k-2MW
                    const float E1 = H(e1, e), E2 = H(e2, e), E3 = H(e3, e);
                    const float Q2r = H(ER + x2, e), Q2i = H(ER + XR + x2, e);
                    H(e0, e) = SE; H(ER + x2, e) = SQR; H(ER + XR + x2, e) = SQI;
                    const float Rm = SE + E1 + E2;
                    const float Rs = Rm + E3;
                    const float Pmr = SQR + Q2r, Pmi = -(SQI + Q2i);
                    const float Psr = SHR, Psi = -SHI;
                    const float ds = fmaxf(Rs, 1e-12f), dm = fmaxf(Rm, 1e-12f);
                    oMs[e] = fmaf(Psr, Psr, Psi * Psi) / (ds * ds);
                    oMm[e] = (fmaxf(Pmr, 0.f) * fmaxf(Pmr, 0.f)) / (dm * dm);
                    oRs[e] = Rs; oRm[e] = Rm; oPsr[e] = Psr; oPsi[e] = Psi; oPmr[e] = Pmr; oPmi[e] = Pmi;
                }
                chR[soh] = CHR + ph_r.tot; chI[soh] = CHI + ph_i.tot;
                cqR[soq] = CQR + pq_r.tot; cqI[soq] = CQI + pq_i.tot; ceE[soq] = CEE + pe.tot;
                CHR += ph_r.tot; CHI += ph_i.tot; CQR += pq_r.tot; CQI += pq_i.tot; CEE += pe.tot;
                const int64_t d0 = nb - (N - 1);
                auto put = [&](float* Mo, float2* Po, float* Ro, const float (&m)[E], const float (&pr)[E],
                               const float (&pi)[E], const float (&r)[E]) {
                    // null outputs stay null (offset only the requested ones)
                    if (Mo) Mo += b * nout;
                    if (Po) Po += b * nout;
                    if (Ro) Ro += b * nout;
#if OFS_SCM_ALIGN == 2
                    if constexpr (E == 4) {                // whole row: 16-byte-aligned stores
                        const int64_t r0 = (int64_t)RL * k - (N - 1);   // d of lane 0, element 0
                        if (r0 >= 0 && r0 + RL <= nout) {               // wave-uniform
                            if (Mo) store_al4(Mo + r0, m, lane);
                            if (Ro) store_al4(Ro + r0, r, lane);
                            if (Po) store_al2(Po + r0, pr, pi, lane);
                            return;
                        }
                    }
#endif
                    if (d0 >= 0 && d0 + E <= nout) {
                        if constexpr (E >= 4) {
                            if (OFS_SCM_ALIGN == 1) {              // 16-byte aligned (row shift s)
#pragma unroll
                                for (int j = 0; j < E; j += 4) {
                                    if (Mo) *reinterpret_cast<float4*>(Mo + d0 + j) = make_float4(m[j], m[j + 1], m[j + 2], m[j + 3]);
                                    if (Ro) *reinterpret_cast<float4*>(Ro + d0 + j) = make_float4(r[j], r[j + 1], r[j + 2], r[j + 3]);
                                }
                            } else {
#pragma unroll
                                for (int j = 0; j < E; j += 2) {
                                    if (Mo) *reinterpret_cast<wf2u*>(Mo + d0 + j) = wf2u{m[j], m[j + 1]};
                                    if (Ro) *reinterpret_cast<wf2u*>(Ro + d0 + j) = wf2u{r[j], r[j + 1]};
                                }
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < E; j += 2) {
                                if (Mo) *reinterpret_cast<wf2u*>(Mo + d0 + j) = wf2u{m[j], m[j + 1]};
                                if (Ro) *reinterpret_cast<wf2u*>(Ro + d0 + j) = wf2u{r[j], r[j + 1]};
                            }
                        }
#pragma unroll
                        for (int j = 0; j < E; j += 2)
                            if (Po) *reinterpret_cast<wf4u*>(Po + d0 + j) = wf4u{pr[j], pi[j], pr[j + 1], pi[j + 1]};
                    } else {
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int64_t d = d0 + e;
                            if (d >= 0 && d < nout) {
                                if (Mo) Mo[d] = m[e];
                                if (Po) Po[d] = make_float2(pr[e], pi[e]);
                                if (Ro) Ro[d] = r[e];
                            }
                        }
                    }
                };
                put(a.Ms, a.Ps, a.Rs, oMs, oPsr, oPsi, oRs);
                put(a.Mm, a.Pm, a.Rm, oMm, oPmr, oPmi, oRm);
            }
        }
    }
}


// Packed form of the fused kernel (OFS_SCM_PK, default): every complex quantity (the x ring, the
// lag-2Q / lag-Q products, their in-lane partials, suffixes and window sums) is one 2 x fp32
// register pair, so products, partials and window sums issue as v_pk_fma / v_pk_mul / v_pk_add
// (half the VALU of the scalar form); the products are formed conjugated, conj(x[j])·x[j-D], so
// P = Σ conj(a) needs no negation; both metrics share one packed multiply by rcp(R²) (1 ulp)
// instead of two IEEE divisions.  Same cancellation-free window split and fp64 row scans.
#ifndef OFS_SCM_PK
#define OFS_SCM_PK 1
#endif

template <int E, int MW, int NB>
__global__ OFS_SCM_BOUNDS void sc_minn_pk_kernel(WinFusedArgs a) {
    constexpr int RL = 64 * E;
    constexpr int N = 4 * MW * RL;
    constexpr int XR = 2 * MW;                  // x ring / S_h suffix ring / S_q history ring
    constexpr int ER = 4 * MW;                  // S_e history ring
    constexpr int PD = 2;
    constexpr int PER = ER;
    constexpr int V4 = E / 2;
    constexpr int WG = scm_wg(NB);
    __shared__ float histE[WG / 64][ER][E][64];     // S_e of the last ER rows
    __shared__ pf2 histQ[WG / 64][XR][E][64];       // conj S_q of the last XR rows
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t b = (int64_t)xcd_block_w() * (WG / 64) + w;
    if (b >= a.B) return;
    const int64_t T = a.T;
    const int64_t nout = T - N + 1;
    const int nrows = (int)((T + RL - 1) / RL);
    const float2* xb = reinterpret_cast<const float2*>(a.x) + b * NB * T;   // [NB][T] of stream b

    pf2 xq[NB][XR][E];                          // x of rows k-2MW..k-1
    pf2 shS[XR][E];                             // S_h suffixes (window 2Q = XR rows)
    pf2 sqS[MW][E];                             // S_q suffixes (window Q = MW rows)
    float seE[MW][E];                           // S_e suffixes
    double chR[XR], chI[XR], cqR[MW], cqI[MW], ceE[MW];
    double CHR = 0, CHI = 0, CQR = 0, CQI = 0, CEE = 0;
#pragma unroll
    for (int m = 0; m < XR; ++m) {
        chR[m] = 0; chI[m] = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            shS[m][e] = pf2{0.f, 0.f};
#pragma unroll
            for (int t = 0; t < NB; ++t) xq[t][m][e] = pf2{0.f, 0.f};
        }
    }
#pragma unroll
    for (int m = 0; m < MW; ++m) {
        cqR[m] = 0; cqI[m] = 0; ceE[m] = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) { sqS[m][e] = pf2{0.f, 0.f}; seE[m][e] = 0.f; }
    }

    float4 nx[PD][NB][V4];
    // whole rows as 8-byte-aligned float4 pairs; the last, partial row per sample, zeros past T
    auto load_row = [&](int k, float4 (&dst)[NB][V4]) {
        const int64_t n0 = (int64_t)RL * k + E * lane;
        const bool whole = (int64_t)RL * (k + 1) <= T;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const float2* xs = xb + (int64_t)t * T;
#pragma unroll
            for (int j = 0; j < V4; ++j) {
                if (whole) {
                    const wf4u v = *reinterpret_cast<const wf4u*>(xs + n0 + 2 * j);
                    dst[t][j] = make_float4(v.x, v.y, v.z, v.w);
                } else {
                    const int64_t m0 = n0 + 2 * j;
                    const float2 u0 = m0 < T ? xs[m0] : make_float2(0.f, 0.f);
                    const float2 u1 = m0 + 1 < T ? xs[m0 + 1] : make_float2(0.f, 0.f);
                    dst[t][j] = make_float4(u0.x, u0.y, u1.x, u1.y);
                }
            }
        }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) load_row(p < nrows ? p : 0, nx[p]);

    for (int k0 = 0; k0 < nrows; k0 += PER) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = k0 + u;
            if (k < nrows) {
                const int x2 = u % XR;                 // row k-2MW (x ring), then row k
                const int x1 = (u + MW) % XR;          // row k-MW
                pf2 h[E], q[E];
                float en[E];
#pragma unroll
                for (int e = 0; e < E; ++e) { h[e] = pf2{0.f, 0.f}; q[e] = pf2{0.f, 0.f}; en[e] = 0.f; }
#pragma unroll
                for (int t = 0; t < NB; ++t) {         // products summed over the branches
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const float4 v = nx[u % PD][t][e / 2];
                        const pf2 c = (e & 1) ? pf2{v.z, v.w} : pf2{v.x, v.y};
                        en[e] += fmaf(c.x, c.x, c.y * c.y);
                        h[e] = cjmul_acc(c, xq[t][x2][e], h[e]);
                        q[e] = cjmul_acc(c, xq[t][x1][e], q[e]);
                        xq[t][x2][e] = c;
                    }
                }
                if (k + PD < nrows) load_row(k + PD, nx[u % PD]);
                // in-lane forward / backward partials, fp64 wave scans of the lane totals
                pf2 fh[E], gh[E], fq[E], gq[E];
                float fe[E], ge[E];
                fh[0] = h[0]; fq[0] = q[0]; fe[0] = en[0];
#pragma unroll
                for (int e = 1; e < E; ++e) { fh[e] = fh[e - 1] + h[e]; fq[e] = fq[e - 1] + q[e]; fe[e] = fe[e - 1] + en[e]; }
                gh[E - 1] = pf2{0.f, 0.f}; gq[E - 1] = pf2{0.f, 0.f}; ge[E - 1] = 0.f;
#pragma unroll
                for (int e = E - 2; e >= 0; --e) { gh[e] = gh[e + 1] + h[e + 1]; gq[e] = gq[e + 1] + q[e + 1]; ge[e] = ge[e + 1] + en[e + 1]; }
                const double ihR = scan_add((double)fh[E - 1].x), ihI = scan_add((double)fh[E - 1].y);
                const double iqR = scan_add((double)fq[E - 1].x), iqI = scan_add((double)fq[E - 1].y);
                const double ie = scan_add((double)fe[E - 1]);
                const double thR = readlane(ihR, 63), thI = readlane(ihI, 63);
                const double tqR = readlane(iqR, 63), tqI = readlane(iqI, 63), te = readlane(ie, 63);
                const pf2 xh = pf2{(float)shr1z(ihR), (float)shr1z(ihI)}, uh = pf2{(float)(thR - ihR), (float)(thI - ihI)};
                const pf2 xqq = pf2{(float)shr1z(iqR), (float)shr1z(iqI)}, uq = pf2{(float)(tqR - iqR), (float)(tqI - iqI)};
                const float xe = (float)shr1z(ie), ue = (float)(te - ie);
                const int sq = u % MW, soq = (u + 1) % MW, soh = (u + 1) % XR;
                const pf2 wh = k >= XR ? pf2{(float)(CHR - chR[soh]), (float)(CHI - chI[soh])} : pf2{(float)CHR, (float)CHI};
                const pf2 wq = k >= MW ? pf2{(float)(CQR - cqR[soq]), (float)(CQI - cqI[soq])} : pf2{(float)CQR, (float)CQI};
                const float we = (float)(k >= MW ? CEE - ceE[soq] : CEE);
                const int e0 = u % ER, e1 = (u + 3 * MW) % ER, e2 = (u + 2 * MW) % ER, e3 = (u + MW) % ER;
                float oMs[E], oRs[E], oMm[E], oRm[E];
                pf2 oPs[E], oPm[E];
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    pf2 SH = wh + (xh + fh[e]), SQ = wq + (xqq + fq[e]);
                    float SE = we + (xe + fe[e]);
                    if (k >= XR) SH += shS[x2][e];
                    if (k >= MW) { SQ += sqS[sq][e]; SE += seE[sq][e]; }
                    shS[x2][e] = uh + gh[e];
                    sqS[sq][e] = uq + gq[e];
                    seE[sq][e] = ue + ge[e];
                    // histories (LDS): S_e rows k-MW, k-2MW, k-3MW; S_q row k-2MW
                    const float E1 = histE[w][e1][e][lane], E2 = histE[w][e2][e][lane], E3 = histE[w][e3][e][lane];
                    const pf2 Q2 = histQ[w][x2][e][lane];
                    histE[w][e0][e][lane] = SE;
                    histQ[w][x2][e][lane] = SQ;
                    const float Rm = SE + E1 + E2;
                    const float Rs = Rm + E3;
                    const pf2 Pm = SQ + Q2;
                    const float ds = fmaxf(Rs, 1e-12f), dm = fmaxf(Rm, 1e-12f);
                    const pf2 d2 = pf2{ds, dm} * pf2{ds, dm};
                    const float pmr = fmaxf(Pm.x, 0.f);
                    const pf2 num = pf2{fmaf(SH.x, SH.x, SH.y * SH.y), pmr * pmr};
                    const pf2 mm = num * pf2{__builtin_amdgcn_rcpf(d2.x), __builtin_amdgcn_rcpf(d2.y)};
                    oMs[e] = mm.x; oMm[e] = mm.y; oRs[e] = Rs; oRm[e] = Rm; oPs[e] = SH; oPm[e] = Pm;
                }
                chR[soh] = CHR + thR; chI[soh] = CHI + thI;
                cqR[soq] = CQR + tqR; cqI[soq] = CQI + tqI; ceE[soq] = CEE + te;
                CHR += thR; CHI += thI; CQR += tqR; CQI += tqI; CEE += te;
                const int64_t d0 = (int64_t)RL * k + E * lane - (N - 1);
                auto put = [&](float* Mo, float2* Po, float* Ro, const float (&m)[E], const pf2 (&pp)[E], const float (&r)[E]) {
                    if (Mo) Mo += b * nout;
                    if (Po) Po += b * nout;
                    if (Ro) Ro += b * nout;
                    if (d0 >= 0 && d0 + E <= nout) {
#pragma unroll
                        for (int j = 0; j < E; j += 2) {
                            if (Mo) *reinterpret_cast<wf2u*>(Mo + d0 + j) = wf2u{m[j], m[j + 1]};
                            if (Ro) *reinterpret_cast<wf2u*>(Ro + d0 + j) = wf2u{r[j], r[j + 1]};
                            if (Po) *reinterpret_cast<wf4u*>(Po + d0 + j) = wf4u{pp[j].x, pp[j].y, pp[j + 1].x, pp[j + 1].y};
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int64_t d = d0 + e;
                            if (d >= 0 && d < nout) {
                                if (Mo) Mo[d] = m[e];
                                if (Po) Po[d] = make_float2(pp[e].x, pp[e].y);
                                if (Ro) Ro[d] = r[e];
                            }
                        }
                    }
                };
                put(a.Ms, a.Ps, a.Rs, oMs, oPs, oRs);
                put(a.Mm, a.Pm, a.Rm, oMm, oPm, oRm);
            }
        }
    }
}

template <int MODE, int E, int MW, int NB>
int launch(const WinFastArgs& a, hipStream_t st) {
    const int64_t grid = (a.B + WF_WG / 64 - 1) / (WF_WG / 64);
    hipLaunchKernelGGL((win_fast_kernel<MODE, E, MW, NB>), dim3((unsigned)grid), dim3(WF_WG), ofs::occ_lds(), st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

template <int MODE, int E, int NB>
int launch_mw(int mw, const WinFastArgs& a, hipStream_t st) {
    switch (mw) {
        case 1: return launch<MODE, E, 1, NB>(a, st);
        case 2: return launch<MODE, E, 2, NB>(a, st);
        case 4: return launch<MODE, E, 4, NB>(a, st);
        case 8: return launch<MODE, E, 8, NB>(a, st);
    }
    return 0;
}

template <int MODE, int NB>
int launch_e(int e, int mw, const WinFastArgs& a, hipStream_t st) {
    switch (e) {
        case 2: return launch_mw<MODE, 2, NB>(mw, a, st);
        case 4: return launch_mw<MODE, 4, NB>(mw, a, st);
    }
    return 0;
}

// samples per lane per row E and window rows MW for window W, or E = 0 if not covered
void pick(int W, int& E, int& mw) {
    // prefer short register rings (MW <= 4), then wider rows
    E = 0; mw = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int e : {4, 2}) {
            const int rl = 64 * e;
            if (W % rl) continue;
            const int m = W / rl;
            if ((pass == 0 && (m == 1 || m == 2 || m == 4)) || (pass == 1 && m == 8)) { E = e; mw = m; return; }
        }
}

template <int E, int MW, int NB>
int launch_fused(const WinFusedArgs& a, hipStream_t st) {
    constexpr int WG = scm_wg(NB);
    const int64_t grid = (a.B + WG / 64 - 1) / (WG / 64);
    if (OFS_SCM_PK)
        hipLaunchKernelGGL((sc_minn_pk_kernel<E, MW, NB>), dim3((unsigned)grid), dim3(WG), ofs::occ_lds(), st, a);
    else
        hipLaunchKernelGGL((sc_minn_fast_kernel<E, MW, NB>), dim3((unsigned)grid), dim3(WG), ofs::occ_lds(), st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

}  // namespace

int ofs_sc_minn_fast_plan(int fmt, int precision, int n_br, int64_t T, int N) {
    if (fmt != OFS_C64 || precision != OFS_FP32 || n_br < 1 || n_br > 2 || T < N || N % 4) return 0;
    const int Q = N / 4;
    for (int e : {4, 2}) {                     // per-wave LDS history: 64·E·(8·MW) floats
        if (Q % (64 * e)) continue;
        const int m = Q / (64 * e);
        if (m == 1 || m == 2 || (m == 4 && e == 2)) return 10 * e + m;
    }
    return 0;
}

int ofs_sc_minn_fast_try(int fmt, int precision, int n_br, const void* x, int64_t B, int64_t T, int N,
                         void* Ms, void* Ps, void* Rs, void* Mm, void* Pm, void* Rm, hipStream_t st) {
    const int plan = ofs_sc_minn_fast_plan(fmt, precision, n_br, T, N);
    if (!plan) return 0;
    const WinFusedArgs a{x, B, T, N, (float*)Ms, (float2*)Ps, (float*)Rs, (float*)Mm, (float2*)Pm, (float*)Rm};
    if (n_br == 2) {
        switch (plan) {
            case 41: return launch_fused<4, 1, 2>(a, st);
            case 42: return launch_fused<4, 2, 2>(a, st);
            case 21: return launch_fused<2, 1, 2>(a, st);
            case 22: return launch_fused<2, 2, 2>(a, st);
            default: return launch_fused<2, 4, 2>(a, st);
        }
    }
    switch (plan) {
        case 41: return launch_fused<4, 1, 1>(a, st);
        case 42: return launch_fused<4, 2, 1>(a, st);
        case 21: return launch_fused<2, 1, 1>(a, st);
        case 22: return launch_fused<2, 2, 1>(a, st);
        default: return launch_fused<2, 4, 1>(a, st);
    }
}

int ofs_win_fast_plan(int mode, int fmt, int precision, int n_br, int64_t T, int N) {
    if (fmt != OFS_C64 || precision != OFS_FP32 || n_br < 1 || n_br > 2 || T < N) return 0;
    if (mode < WF_SC || mode > WF_MINN) return 0;
    const int div = mode == WF_MINN ? 4 : 2;
    if (N % div) return 0;
    int E, mw;
    pick(N / div, E, mw);
    if (n_br == 2 && mw == 8) return 0;         // the two-branch x ring would spill (general engine)
    return E ? 10 * E + mw : 0;
}

int ofs_win_fast_try(int mode, int fmt, int precision, int n_br, const WinFastArgs& a, hipStream_t st) {
    const int plan = ofs_win_fast_plan(mode, fmt, precision, n_br, a.T, a.N);
    if (!plan) return 0;
    const int E = plan / 10, mw = plan % 10;
    if (n_br == 2) {
        switch (mode) {
            case WF_SC: return launch_e<WF_SC, 2>(E, mw, a, st);
            case WF_COMB: return launch_e<WF_COMB, 2>(E, mw, a, st);
            default: return launch_e<WF_MINN, 2>(E, mw, a, st);
        }
    }
    switch (mode) {
        case WF_SC: return launch_e<WF_SC, 1>(E, mw, a, st);
        case WF_COMB: return launch_e<WF_COMB, 1>(E, mw, a, st);
        default: return launch_e<WF_MINN, 1>(E, mw, a, st);
    }
}
