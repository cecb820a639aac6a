// aa_fast.hip — register-resident fast path of the [A][A] S&C detector (sync_aa.py:421-571).
//
// One wave64 per receive stream, no LDS, no barriers.  Row k of a stream holds RL = 64·E
// samples; lane l owns the E consecutive samples n = RL·k + E·l + e.  With L = MR·RL the
// delayed sample x[n-L] sits in the SAME lane and element MR rows back, so the lagged
// product x[n]·conj(x[n-L]) needs no data movement.
//
// Window sums without cancellation: for n in row k (k >= MR)
//     P[n] = suf_{k-MR}(e') + sum_{j=k-MR+1}^{k-1} tot_j + pre_k(e')
// where pre_k is the in-row inclusive prefix (fp64: lane-serial + DPP wave scan), tot_j the
// row totals (fp64, wave-uniform) and suf_{k-MR} the part of row k-MR after position n —
// computed in fp64 when that row was processed and retained in fp32 registers.  Every piece
// sums only in-window terms, so fp32 storage error is relative to the window, not to the
// stream or a loud burst next to a quiet window.  Each row is processed in two passes:
// (1) lane totals -> wave scan; (2) products recomputed while outputs stream out, which keeps
// the register footprint at ~3L/64 retained floats per lane.
//
// Gate / peak / CFO events (sync_aa.py:495-568) use the closed form of aa_events
// (ofdmsync.hip), streamed row by row (aa_gate.h): prev-above by lane-serial + DPP max-scan,
// opens/closes by ballot, per-gate argmax by wave reductions, scalar carry between rows.
#include "ofs_common.h"
#include "aa_gate.h"
#include "ofdmsync.h"

using namespace ofs;

namespace {

#ifndef OFS_FAST_WG
#define OFS_FAST_WG 64
#endif
constexpr int FAST_WG = OFS_FAST_WG;   // one wave = one stream per workgroup (paired A/B: 2-6 % faster than 256)

// occupancy bound (min waves per SIMD) of the fast kernel; tuning builds set -DOFS_FAST_WAVES=N
#ifndef OFS_FAST_WAVES
#define OFS_FAST_WAVES 0
#endif
#if OFS_FAST_WAVES > 0
#define OFS_FAST_BOUNDS __launch_bounds__(FAST_WG, OFS_FAST_WAVES)
#else
#define OFS_FAST_BOUNDS __launch_bounds__(FAST_WG)
#endif
constexpr int TMAX = 1024;        // stream length handled by the fast path
constexpr int FAST_CAP_LDS = 160 * 1024 / 10;   // occupancy cap of the storing kernel: 10 workgroups per CU (launch)

// cache policy knobs (tuning builds): non-temporal output stores, LDS-DMA aux bits
#ifndef OFS_STORE_NT
#define OFS_STORE_NT 0
#endif
#ifndef OFS_DMA_AUX
#define OFS_DMA_AUX 0
#endif
// stream staging: 0 = LDS-DMA (global_load_lds_dwordx4), 1 = registers, 2 = registers with the loads
// pinned as inline asm + per-row vmcnt waits (tuning builds; r06b below)
#ifndef OFS_FAST_STAGE
#define OFS_FAST_STAGE 1
#endif
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef float nf2 __attribute__((ext_vector_type(2)));
// complex values as packed fp32 pairs (re, im): products, in-lane partials and window sums issue
// as v_pk_fma / v_pk_add (half the VALU of the scalar form)
typedef float pf2 __attribute__((ext_vector_type(2)));
// acc + c·conj(d) = acc + (c.x d.x + c.y d.y, c.y d.x - c.x d.y)
__device__ __forceinline__ pf2 mulc_acc(pf2 c, pf2 d, pf2 acc) {
    acc = __builtin_elementwise_fma(c, d.xx, acc);
    return __builtin_elementwise_fma(c.yx, pf2{d.y, -d.y}, acc);
}
__device__ __forceinline__ void st_out(float4* p, float4 v) {
#if OFS_STORE_NT
    __builtin_nontemporal_store(nf4{v.x, v.y, v.z, v.w}, reinterpret_cast<nf4*>(p));
#else
    *p = v;
#endif
}
__device__ __forceinline__ void st_out(float2* p, float2 v) {
#if OFS_STORE_NT
    __builtin_nontemporal_store(nf2{v.x, v.y}, reinterpret_cast<nf2*>(p));
#else
    *p = v;
#endif
}


// Stream staging (OFS_FAST_STAGE): 1 (default) = every row of the lane's samples is loaded into
// registers up front, each row's first use waits only for its own loads; 0 = the wave DMAs its
// stream into a private 8 KiB LDS slice (global_load_lds_dwordx4) and reads rows back with
// ds_read_b128.  Paired A/B on the same buffers: registers 1-3 % faster (profiles/
// r01c_staging_ab.log; the SOL probe shows the same 8 % gap between LDS-DMA and register staging
// of this read/write pattern).  Round 2, with the DMA as inline asm and per-row vmcnt waits (the
// builtin made the compiler wait for the whole stream before the first row) and 107 instead of
// 139 VGPRs (4 waves/SIMD): still 3 % slower (0.315 vs 0.305 ms, profiles/r02av_staging_ab.jsonl).
// Round 6, the loads pinned (OFS_FAST_STAGE=2: inline-asm global_load_dwordx4, per-row vmcnt) so a
// tight register budget cannot defer them: 105 VGPRs at 4 waves/SIMD, no spills, bit-identical - and
// more waves are SLOWER, not faster (paired, 9 rotated rounds, profiles/r06b_headline_pinned_loads_
// waves_ab.jsonl): 3 waves 0.3067 ms (plain) / 0.3082 (pinned), 4 waves 0.3150 (pinned) / 0.3137
// (plain), 5 waves 0.3283 (pinned).  The kernel is not latency-starved at 3 waves/SIMD.
// scan-free gate flags in the P/R/M-storing instantiation too (tuning builds: -DOFS_FAST_FF=1)
#ifndef OFS_FAST_FF
#define OFS_FAST_FF 0
#endif
// tuning builds: 1 = gate machine after the row loop - each row's (M, |P|^2, P) of the gated rows goes to
// a wave-private LDS slice and the gate runs over them once every row's stores have issued.  Measured
// (paired, profiles/r05_headline_gate_breakdown.txt): neutral on the headline (0.2937-0.3053 vs
// 0.2924-0.3056 ms), 5 % slower detect-only (0.107 vs 0.102 ms); default 0 = per row
#ifndef OFS_FAST_GATE_LATE
#define OFS_FAST_GATE_LATE 0
#endif
// DO: detect-only instantiation (P/R/M/valid not stored, events only: SURVEY §8d); S32: fp32
// row scans (ofs_common.h row_scan; the detect-only default, issue-bound there)
template <int E, int MR, int NA, bool DO, bool S32>
__global__ OFS_FAST_BOUNDS void aa_fast_kernel(AaFastArgs a) {
    constexpr int RL = 64 * E;                 // samples per row
    constexpr int RW = TMAX / RL;              // rows per stream
    constexpr int L = MR * RL;
    constexpr int V4 = E / 2;                  // float4 (2 samples) per lane per row
    static_assert(MR >= 1 && MR <= RW, "window must fit the stream tile");
#if OFS_FAST_STAGE == 0
    __shared__ float4 lds[FAST_WG / 64][NA * RW * V4][64];
#endif
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    // block order: one antenna plain blockIdx, two the XCD remap (paired under the occupancy cap,
    // profiles/r06n_headline_remap_ff_ab.txt: without the remap cfg3 0.2994 -> 0.2940 ms, detect-only
    // 0.1036 -> 0.0949, T 4096 1.225 -> 1.211; two antennas 0.4004 -> 0.4055 and the 2 x 5315 shape
    // slower in 2 of 3 rounds - they keep it)
    const int64_t b = (int64_t)(NA == 1 ? blockIdx.x : xcd_block()) * (FAST_WG / 64) + w;
    if (b >= a.B) return;
    const int T = (int)a.T;
#if OFS_FAST_STAGE == 0
    // row-major DMA order (row k of every antenna before row k+1): row k has landed once at most
    // the later rows' DMAs and the output stores of rows < k (SPR per row, all younger) are
    // outstanding - vmcnt counts in order.  The DMA goes through inline asm (ofs::lds_dma16): the
    // builtin makes the compiler wait for every DMA before the first LDS read.  Event stores are
    // not counted (a larger count could only under-wait; a smaller one waits longer).
    constexpr int SPR = V4 + ((E % 4 != 0) ? 2 * V4 : 2 * (V4 / 2));   // P + R + M stores per row
#pragma unroll
    for (int k = 0; k < RW; ++k)
#pragma unroll
        for (int t = 0; t < NA; ++t) {
            const float2* xs = reinterpret_cast<const float2*>(a.x) + (b * NA + t) * a.T;
#pragma unroll
            for (int j = 0; j < V4; ++j) {
                int n = RL * k + E * lane + 2 * j;
                n = n < T ? n : T - 2;                          // in-bounds; zeroed on read
                ofs::lds_dma16(xs + n, &lds[w][(t * RW + k) * V4 + j][0]);
            }
        }
    auto ldrow = [&](int t, int k, int j) { return lds[w][(t * RW + k) * V4 + j][lane]; };
    // SPR counts only when all of P, R, M are stored (uncounted stores only make the wait longer)
    const bool all_out = !DO && a.P && a.R && a.M;
    auto row_wait = [&](int k) {
        if (all_out) ofs::vmcnt_wait((RW - 1 - k) * NA * V4 + k * SPR);
        else ofs::vmcnt_wait((RW - 1 - k) * NA * V4);
    };
#elif OFS_FAST_STAGE == 2
    // register staging with the loads PINNED at the top: each load is an inline-asm
    // global_load_dwordx4 (the compiler cannot sink it under a tight register budget, which is
    // what the plain loads did at 4 waves/SIMD), each row's first use waits with its own
    // s_waitcnt vmcnt(n) - n = the younger operations still allowed in flight, vmcnt counting
    // in order: the loads of later rows, plus, for a full stream (T = TMAX, every row's stores
    // issued by every lane) with P, R and M all stored, the SPR stores of each earlier row.  Any
    // other shape counts the loads alone (the stores then only lengthen the wait).  An empty asm
    // that rewrites the row's registers right after the wait keeps their uses behind it.
    constexpr int SPR = V4 + ((E % 4 != 0) ? 2 * V4 : 2 * (V4 / 2));   // P + R + M stores per row
    nf4 xreg[NA][RW][V4];
#pragma unroll
    for (int k = 0; k < RW; ++k)
#pragma unroll
        for (int t = 0; t < NA; ++t) {
            const float2* xs = reinterpret_cast<const float2*>(a.x) + (b * NA + t) * a.T;
#pragma unroll
            for (int j = 0; j < V4; ++j) {
                int n = RL * k + E * lane + 2 * j;
                n = n < T ? n : T - 2;                          // in-bounds; zeroed on read
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(xreg[t][k][j]) : "v"(xs + n) : "memory");
            }
        }
    const bool count_st = !DO && a.P && a.R && a.M && T == TMAX;
    auto ldrow = [&](int t, int k, int j) { const nf4 v = xreg[t][k][j]; return make_float4(v.x, v.y, v.z, v.w); };
    auto row_wait = [&](int k) {
        if (count_st) ofs::vmcnt_wait((RW - 1 - k) * NA * V4 + k * SPR);
        else ofs::vmcnt_wait((RW - 1 - k) * NA * V4);
#pragma unroll
        for (int t = 0; t < NA; ++t)
#pragma unroll
            for (int j = 0; j < V4; ++j) asm volatile("" : "+v"(xreg[t][k][j]));
    };
#else
    // register staging: every row of the lane's samples is loaded up front (RW * V4 float4), each
    // row's first use waits only for its own loads (vmcnt counts in order)
    float4 xreg[NA][RW][V4];
#pragma unroll
    for (int t = 0; t < NA; ++t) {
        const float2* xs = reinterpret_cast<const float2*>(a.x) + (b * NA + t) * a.T;
#pragma unroll
        for (int k = 0; k < RW; ++k)
#pragma unroll
            for (int j = 0; j < V4; ++j) {
                int n = RL * k + E * lane + 2 * j;
                n = n < T ? n : T - 2;                          // in-bounds; zeroed on read
                xreg[t][k][j] = *reinterpret_cast<const float4*>(xs + n);
            }
    }
    auto ldrow = [&](int t, int k, int j) { return xreg[t][k][j]; };
    auto row_wait = [&](int) {};
#endif
    auto xrow = [&](int t, int k, pf2 (&c)[E]) {
#pragma unroll
        for (int j = 0; j < V4; ++j) {
            const bool ok = RL * k + E * lane + 2 * j < T;
            const float4 v = ldrow(t, k, j);
            c[2 * j] = ok ? pf2{v.x, v.y} : pf2{0.f, 0.f};
            c[2 * j + 1] = ok ? pf2{v.z, v.w} : pf2{0.f, 0.f};
        }
    };

    pf2 sS[MR][E];                              // retained in-window suffixes (ring by k % MR)
    float sE[MR][E];
    double Cr[RW + 1], Ci[RW + 1], Ce[RW + 1];  // running row bases (wave-uniform)
    Cr[0] = Ci[0] = Ce[0] = 0.0;

    // scan-free gate flags: detect-only, and the one-antenna storing kernel (round 6, under the occupancy
    // cap: 0.2905 -> 0.2889 ms, 0.2979 -> 0.2966 with the remap; r06m / r06n)
    AaRowGate<E, float, false, (bool)(DO || OFS_FAST_FF || NA == 1)> gate;   // event state (wave-uniform)
#if OFS_FAST_GATE_LATE
    constexpr int GR = RW - MR > 0 ? RW - MR : 1;             // gated rows (k >= MR)
    __shared__ float4 gl[FAST_WG / 64][GR][E][64];            // (M, |P|^2, Re P, Im P) per sample
#endif
    if (a.detect)
        gate.init(a.hyst, L, a.thr, a.fs, a.max_ev, a.ev_i + b * (int64_t)a.max_ev * 4,
                  a.ev_r + b * (int64_t)a.max_ev * 4);

    float* Pout = DO ? nullptr : reinterpret_cast<float*>(a.P);
    float* Rout = DO ? nullptr : reinterpret_cast<float*>(a.R);
    float* Mout = DO ? nullptr : reinterpret_cast<float*>(a.M);
    const float floor_ = 1e-6f * (float)L;

#pragma unroll
    for (int k = 0; k < RW; ++k) {
        if (RL * k < T) {                                       // wave-uniform row guard
            const int nb = RL * k + E * lane;                   // first sample of this lane
            // ---- lagged products x[n]·conj(x[n-L]) and energies, fp32 ----
            // summed over the antennas, like the reference's per-antenna running sums added up
            // (sync_aa.py:463-480)
            pf2 av[E];
            float aE[E];
#pragma unroll
            for (int e = 0; e < E; ++e) { av[e] = pf2{0.f, 0.f}; aE[e] = 0.f; }
            row_wait(k);
#pragma unroll
            for (int t = 0; t < NA; ++t) {
                pf2 c[E];
                xrow(t, k, c);
#pragma unroll
                for (int e = 0; e < E; ++e) aE[e] += fmaf(c[e].x, c[e].x, c[e].y * c[e].y);
                if (k >= MR) {
                    pf2 d[E];
                    xrow(t, k - MR, d);
#pragma unroll
                    for (int e = 0; e < E; ++e) av[e] = mulc_acc(c[e], d[e], av[e]);
                }
            }
            // ---- in-lane partials, each summing only the terms it stands for:
            //      forward f[e] = sum_{e'<=e} a[e'], backward g[e] = sum_{e'>e} a[e'] ----
            pf2 fS[E], gS[E];
            float fE[E], gE[E];
            fS[0] = av[0]; fE[0] = aE[0];
#pragma unroll
            for (int e = 1; e < E; ++e) { fS[e] = fS[e - 1] + av[e]; fE[e] = fE[e - 1] + aE[e]; }
            gS[E - 1] = pf2{0.f, 0.f}; gE[E - 1] = 0.f;
#pragma unroll
            for (int e = E - 2; e >= 0; --e) { gS[e] = gS[e + 1] + av[e + 1]; gE[e] = gE[e + 1] + aE[e + 1]; }
            // ---- lane totals: fp64 DPP wave scan, row totals, rows inside the window ----
            const RowScan sRr = row_scan<S32>(fS[E - 1].x), sIr = row_scan<S32>(fS[E - 1].y), sEr = row_scan<S32>(fE[E - 1]);
            const double totR = sRr.tot, totI = sIr.tot, totE = sEr.tot;
            const pf2 xS = pf2{sRr.x, sIr.x};                        // lanes < l
            const float xE = sEr.x;
            const pf2 uS = pf2{sRr.u, sIr.u};                        // lanes > l
            const float uE = sEr.u;
            Cr[k + 1] = Cr[k] + totR; Ci[k + 1] = Ci[k] + totI; Ce[k + 1] = Ce[k] + totE;
            const pf2 wS = pf2{(float)((k >= MR) ? (Cr[k] - Cr[k - MR + 1]) : Cr[k]),
                               (float)((k >= MR) ? (Ci[k] - Ci[k - MR + 1]) : Ci[k])};
            const float wE = (float)((k >= MR) ? (Ce[k] - Ce[k - MR + 1]) : Ce[k]);

            // ---- window sums  P = suffix(row k-MR) + rows between + prefix(row k) ----
            float pf[E][2], mf[E], pmf[E], rf[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                pf2 P = wS + (xS + fS[e]);
                float RR = wE + (xE + fE[e]);
                if (k >= MR) { P += sS[k % MR][e]; RR += sE[k % MR][e]; }
                sS[k % MR][e] = uS + gS[e]; sE[k % MR][e] = uE + gE[e];
                const float pm = fmaf(P.x, P.x, P.y * P.y);
                float m = 0.f;
                if (k >= MR && RR > floor_) m = fminf(pm * __builtin_amdgcn_rcpf(RR * RR), 1.f);
                pf[e][0] = P.x; pf[e][1] = P.y; rf[e] = RR; mf[e] = m; pmf[e] = pm;
            }

            const int64_t o = b * a.T + nb;
#pragma unroll
            for (int j = 0; j < V4; ++j) {
                if (nb + 2 * j < T) {
                    if (Pout) st_out(reinterpret_cast<float4*>(Pout + 2 * (o + 2 * j)),
                                    make_float4(pf[2 * j][0], pf[2 * j][1], pf[2 * j + 1][0], pf[2 * j + 1][1]));
                    // float4 R/M stores need T % 4 == 0: otherwise the last pair of a stream
                    // would spill into the next stream's first samples (and b*T+nb is not
                    // 16-byte aligned for odd b)
                    if (E % 4 != 0 || (T & 3) != 0) {
                        if (Rout) st_out(reinterpret_cast<float2*>(Rout + o + 2 * j), make_float2(rf[2 * j], rf[2 * j + 1]));
                        if (Mout) st_out(reinterpret_cast<float2*>(Mout + o + 2 * j), make_float2(mf[2 * j], mf[2 * j + 1]));
                    } else if ((j & 1) == 0) {
                        if (Rout) st_out(reinterpret_cast<float4*>(Rout + o + 2 * j),
                                        make_float4(rf[2 * j], rf[2 * j + 1], rf[2 * j + 2], rf[2 * j + 3]));
                        if (Mout) st_out(reinterpret_cast<float4*>(Mout + o + 2 * j),
                                        make_float4(mf[2 * j], mf[2 * j + 1], mf[2 * j + 2], mf[2 * j + 3]));
                    }
                    if (!DO && a.valid) { a.valid[o + 2 * j] = (k >= MR); a.valid[o + 2 * j + 1] = (k >= MR); }
                }
            }

            // ---- events: closed-form gate machine, streamed per row (aa_gate.h) ----
            if (a.detect && k >= MR) {
#if OFS_FAST_GATE_LATE
#pragma unroll
                for (int e = 0; e < E; ++e) gl[w][k >= MR ? k - MR : 0][e][lane] = make_float4(mf[e], pmf[e], pf[e][0], pf[e][1]);
#else
                float pr[E], pi[E];
#pragma unroll
                for (int e = 0; e < E; ++e) { pr[e] = pf[e][0]; pi[e] = pf[e][1]; }
                gate.row(lane, k, nb, T, mf, pmf, pr, pi);
#endif
            }
        }
    }
#if OFS_FAST_GATE_LATE
    if (a.detect) {
        // this wave's own LDS slice, written lane-wise above: a wave-local hand-over
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
        for (int k = MR; k < RW; ++k) {
            if (RL * k >= T) break;
            float m[E], pm[E], pr[E], pi[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float4 v = gl[w][k - MR][e][lane];
                m[e] = v.x; pm[e] = v.y; pr[e] = v.z; pi[e] = v.w;
            }
            gate.row(lane, k, RL * k + E * lane, T, m, pm, pr, pi);
        }
    }
#endif
    if (a.detect) gate.finish(lane, T, a.n_ev + b);
}

// ------------------------------------------------------------------------------------------
// Streaming variant for ANY stream length (T > 1024 or odd T: the reference's own detector
// input, sync_aa.run_single_test, is ~4.2-5.3k samples x 2 antennas, sync_aa.py:699-738).
// Same row layout, window split and gate machine as aa_fast_kernel; instead of holding the
// whole stream in registers, rows stream from HBM PD rows ahead of use and only what the
// window needs is retained: the raw samples of rows k-MR..k-1 (lag L = MR rows), the fp32
// in-window suffixes of those rows and the fp64 row bases C[k-MR+1..k] (register rings
// indexed by k mod MR, resolved at compile time by unrolling the row loop by the ring period).
// Odd T: the stream base is only 8-byte aligned, so pair loads/stores use 8-byte-aligned
// vector types (gfx950 global memory ops need dword alignment only) and the last, partial row
// falls back to per-sample accesses.
// ------------------------------------------------------------------------------------------
typedef float f4u __attribute__((ext_vector_type(4), aligned(8)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));

#ifndef OFS_STREAM_WG
#define OFS_STREAM_WG 64
#endif
constexpr int STREAM_WG = OFS_STREAM_WG;
// tuning builds: rows in flight (OFS_STREAM_PD), occupancy bound (OFS_STREAM_WAVES waves/SIMD)
#ifndef OFS_STREAM_PD
#define OFS_STREAM_PD 0
#endif
#ifndef OFS_STREAM_WAVES
#define OFS_STREAM_WAVES 0
#endif
// workgroup size of the streaming kernel: the one-antenna storing kernel runs 2 streams per workgroup
// (round 6, paired, profiles/r06v_stream_kernel_variants_ab.txt: T 4096 1.222 -> 1.192 ms); two
// antennas (the 2 x 5315 reference shape: 0.578 vs 0.608 ms) and detect-only keep one
#ifndef OFS_STREAM_WG1
#define OFS_STREAM_WG1 128
#endif
constexpr int stream_wg(int na, bool det_only) { return (na == 1 && !det_only) ? OFS_STREAM_WG1 : STREAM_WG; }
#if OFS_STREAM_WAVES > 0
#define OFS_STREAM_BOUNDS __launch_bounds__(stream_wg(NA, DO), OFS_STREAM_WAVES)
#else
#define OFS_STREAM_BOUNDS __launch_bounds__(stream_wg(NA, DO))
#endif

#ifndef OFS_STREAM_FF
#define OFS_STREAM_FF 1
#endif
// lag ring (raw samples of rows k-MR..k-1) in a wave-private LDS slice instead of VGPRs:
// 0 = never, 1 = two antennas (frees 32 VGPRs there), 2 = always
#ifndef OFS_STREAM_LDSLAG
#define OFS_STREAM_LDSLAG 1
#endif

// per-wave state of the streaming kernel; row<U, FIRST, GUARD>() processes row k whose ring
// position k mod PER == U is a compile-time constant: FIRST = rows k < MR (no lagged product,
// window clipped at 0), GUARD = a row that may reach past T (partial row / tail)
template <int E, int MR, int NA, bool DO>
struct AaStream {
    static constexpr int RL = 64 * E;
    static constexpr int L = MR * RL;
    static constexpr int V4 = E / 2;                         // sample pairs per lane per row
    // rows in flight ahead of use (paired A/B, tools/lib_ab.py, r02e: 1 antenna PD 2, 2 antennas
    // with the LDS lag ring PD 4; the peeled steady loop + scan-free gate flags + these took the
    // T = 4096 shape 1.32 -> 1.09 ms and the 2 x 5315 reference shape 0.75 -> 0.49 ms)
    static constexpr int PD = OFS_STREAM_PD > 0 ? OFS_STREAM_PD : ((E == 2 && NA == 2) ? 4 : 2);
    static constexpr int PER = MR > PD ? MR : PD;            // unroll period (MR, PD powers of 2)
    static constexpr bool LDSLAG = OFS_STREAM_LDSLAG == 2 || (OFS_STREAM_LDSLAG == 1 && NA == 2);

    const float2* xb;
    float4 (*lag)[NA][V4][64];                               // LDSLAG: [MR][NA][V4][lane]
    int64_t T, o0;
    int Ti, nrows, full_rows, lane;
    pf2 lx[LDSLAG ? 1 : NA][MR][E];                          // x of rows k-MR..k-1 (lag L)
    pf2 sS[MR][E];                                           // retained in-window suffixes
    float sE[MR][E];
    double cbR[MR], cbI[MR], cbE[MR];                        // row bases C[j], j in (k-MR, k]
    double CR, CI, CE;                                       // C[k]: prefix at the start of row k
    float2 nx[PD][NA][E];                                    // rows k..k+PD-1 in flight
    AaRowGate<E, float, false, (bool)(DO || OFS_STREAM_FF)> gate;
    float2* Pout; float* Rout; float* Mout; uint8_t* Vout;
    bool detect;
    float floor_;

    // a row's samples of every antenna: 8-byte-aligned pair loads for whole rows, per-sample
    // with zero fill past T otherwise (wave-uniform choice)
    __device__ __forceinline__ void load_row(int k, float2 (&dst)[NA][E]) {
        const int64_t n0 = (int64_t)RL * k + E * lane;
#pragma unroll
        for (int t = 0; t < NA; ++t) {
            const float2* xs = xb + (int64_t)t * T;
            if (k < full_rows) {
#pragma unroll
                for (int j = 0; j < V4; ++j) {
                    const f4u v = *reinterpret_cast<const f4u*>(xs + n0 + 2 * j);
                    dst[t][2 * j] = make_float2(v.x, v.y);
                    dst[t][2 * j + 1] = make_float2(v.z, v.w);
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) dst[t][e] = (n0 + e < T) ? xs[n0 + e] : make_float2(0.f, 0.f);
            }
        }
    }

    template <int U, bool FIRST, bool GUARD>
    __device__ __forceinline__ void row(int k) {
        constexpr int sl = U % MR;                           // ring slot of row k-MR (and k)
        constexpr int so = (U + 1) % MR;                     // slot of C[k-MR+1]
        const int nb = RL * k + E * lane;
        float2 cur[NA][E];
#pragma unroll
        for (int t = 0; t < NA; ++t)
#pragma unroll
            for (int e = 0; e < E; ++e) cur[t][e] = nx[U % PD][t][e];
        if (!GUARD || k + PD < nrows) load_row(k + PD, nx[U % PD]);
        // lagged samples x[n-L] (row k-MR) of every antenna
        pf2 d[NA][E];
#pragma unroll
        for (int t = 0; t < NA; ++t) {
            if constexpr (LDSLAG) {
#pragma unroll
                for (int j = 0; j < V4; ++j) {
                    const float4 v = FIRST ? make_float4(0.f, 0.f, 0.f, 0.f) : lag[sl][t][j][lane];
                    d[t][2 * j] = pf2{v.x, v.y}; d[t][2 * j + 1] = pf2{v.z, v.w};
                    lag[sl][t][j][lane] = make_float4(cur[t][2 * j].x, cur[t][2 * j].y, cur[t][2 * j + 1].x,
                                                      cur[t][2 * j + 1].y);
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    d[t][e] = lx[t][sl][e];
                    lx[t][sl][e] = pf2{cur[t][e].x, cur[t][e].y};
                }
            }
        }
        // ---- lagged products x[n]·conj(x[n-L]) and energies, summed over the antennas ----
        pf2 av[E];
        float aE[E];
#pragma unroll
        for (int e = 0; e < E; ++e) { av[e] = pf2{0.f, 0.f}; aE[e] = 0.f; }
#pragma unroll
        for (int t = 0; t < NA; ++t)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const pf2 c = pf2{cur[t][e].x, cur[t][e].y};
                aE[e] += fmaf(c.x, c.x, c.y * c.y);
                if (!FIRST) av[e] = mulc_acc(c, d[t][e], av[e]);
            }
        // ---- in-lane partials (forward f, backward g), fp64 wave scan ----
        pf2 fS[E], gS[E];
        float fE[E], gE[E];
        fS[0] = av[0]; fE[0] = aE[0];
#pragma unroll
        for (int e = 1; e < E; ++e) { fS[e] = fS[e - 1] + av[e]; fE[e] = fE[e - 1] + aE[e]; }
        gS[E - 1] = pf2{0.f, 0.f}; gE[E - 1] = 0.f;
#pragma unroll
        for (int e = E - 2; e >= 0; --e) { gS[e] = gS[e + 1] + av[e + 1]; gE[e] = gE[e + 1] + aE[e + 1]; }
        const RowScan se_ = row_scan<false>(fE[E - 1]);
        const double tE = se_.tot;
        const float xE = se_.x, uE = se_.u;
        double tR = 0.0, tI = 0.0;
        pf2 xS = pf2{0.f, 0.f}, uS = pf2{0.f, 0.f};
        if (!FIRST) {                                        // no lagged product before row MR
            const RowScan sr_ = row_scan<false>(fS[E - 1].x), si_ = row_scan<false>(fS[E - 1].y);
            tR = sr_.tot; tI = si_.tot;
            xS = pf2{sr_.x, si_.x};
            uS = pf2{sr_.u, si_.u};
        }
        const pf2 wS = FIRST ? pf2{(float)CR, (float)CI} : pf2{(float)(CR - cbR[so]), (float)(CI - cbI[so])};
        const float wE = (float)(FIRST ? CE : CE - cbE[so]);
        // ---- window sums P = suffix(row k-MR) + rows between + prefix(row k) ----
        float pr[E], pi[E], rf[E], mf[E], pmf[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            pf2 P = wS + (xS + fS[e]);
            float RR = wE + (xE + fE[e]);
            if (!FIRST) { P += sS[sl][e]; RR += sE[sl][e]; }
            sS[sl][e] = uS + gS[e]; sE[sl][e] = uE + gE[e];
            const float pm = fmaf(P.x, P.x, P.y * P.y);
            float m = 0.f;
            if (!FIRST && RR > floor_) m = fminf(pm * __builtin_amdgcn_rcpf(RR * RR), 1.f);
            pr[e] = P.x; pi[e] = P.y; rf[e] = RR; mf[e] = m; pmf[e] = pm;
        }
        cbR[so] = CR + tR; cbI[so] = CI + tI; cbE[so] = CE + tE;
        CR += tR; CI += tI; CE += tE;
        // ---- stores ----
        if (!DO) {
            const int64_t o = o0 + nb;
            if (!GUARD || k < full_rows) {
#pragma unroll
                for (int j = 0; j < V4; ++j) {
                    if (Pout) *reinterpret_cast<f4u*>(Pout + o + 2 * j) = f4u{pr[2 * j], pi[2 * j], pr[2 * j + 1], pi[2 * j + 1]};
                    if (Rout) *reinterpret_cast<f2u*>(Rout + o + 2 * j) = f2u{rf[2 * j], rf[2 * j + 1]};
                    if (Mout) *reinterpret_cast<f2u*>(Mout + o + 2 * j) = f2u{mf[2 * j], mf[2 * j + 1]};
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (nb + e < Ti) {
                        if (Pout) Pout[o + e] = make_float2(pr[e], pi[e]);
                        if (Rout) Rout[o + e] = rf[e];
                        if (Mout) Mout[o + e] = mf[e];
                    }
            }
            if (Vout) {
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (nb + e < Ti) Vout[o + e] = (uint8_t)(!FIRST);
            }
        }
        // ---- events: closed-form gate machine, streamed per row (aa_gate.h) ----
        if (!FIRST && detect) gate.row(lane, k, nb, Ti, mf, pmf, pr, pi);
    }

    // rows [k0, k0 + PER) with k0 % PER == 0; FIRST_BLOCK: k0 == 0 (rows < MR are FIRST)
    template <bool FIRST_BLOCK, bool GUARD, int U = 0>
    __device__ __forceinline__ void block(int k0) {
        if constexpr (U < PER) {
            const int k = k0 + U;
            if (!GUARD || k < nrows) {
                row<U, FIRST_BLOCK && (U < MR), GUARD>(k);
                block<FIRST_BLOCK, GUARD, U + 1>(k0);
            }
        }
    }
};

template <int E, int MR, int NA, bool DO>
__global__ OFS_STREAM_BOUNDS void aa_stream_kernel(AaFastArgs a) {
    using S = AaStream<E, MR, NA, DO>;
    constexpr int SWG = stream_wg(NA, DO);
    __shared__ float4 lagbuf[SWG / 64][S::LDSLAG ? MR : 1][NA][S::V4][64];
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)(NA == 1 ? blockIdx.x : xcd_block()) * (SWG / 64) + (threadIdx.x >> 6);   // (as aa_fast_kernel)
    if (b >= a.B) return;
    S s;
    s.lane = lane;
    s.lag = lagbuf[threadIdx.x >> 6];
    s.T = a.T;
    s.Ti = (int)a.T;
    s.o0 = b * a.T;
    s.nrows = (int)((a.T + S::RL - 1) / S::RL);
    s.full_rows = (int)(a.T / S::RL);                        // rows entirely inside the stream
    s.xb = reinterpret_cast<const float2*>(a.x) + b * NA * a.T;
    s.CR = s.CI = s.CE = 0.0;
#pragma unroll
    for (int m = 0; m < MR; ++m) {
        s.cbR[m] = 0.0; s.cbI[m] = 0.0; s.cbE[m] = 0.0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            s.sS[m][e] = pf2{0.f, 0.f}; s.sE[m][e] = 0.f;
#pragma unroll
            for (int t = 0; t < (S::LDSLAG ? 1 : NA); ++t) s.lx[t][m][e] = pf2{0.f, 0.f};
        }
    }
#pragma unroll
    for (int p = 0; p < S::PD; ++p)
        if (p < s.nrows) s.load_row(p, s.nx[p]);
    s.detect = a.detect != 0;
    if (s.detect)
        s.gate.init(a.hyst, S::L, a.thr, a.fs, a.max_ev, a.ev_i + b * (int64_t)a.max_ev * 4,
                    a.ev_r + b * (int64_t)a.max_ev * 4);
    s.Pout = DO ? nullptr : reinterpret_cast<float2*>(a.P);
    s.Rout = DO ? nullptr : reinterpret_cast<float*>(a.R);
    s.Mout = DO ? nullptr : reinterpret_cast<float*>(a.M);
    s.Vout = DO ? nullptr : a.valid;
    s.floor_ = 1e-6f * (float)S::L;

    // warm-up block (rows 0..PER-1: the first MR have no lagged product), steady blocks of
    // whole rows with no per-row guards, then the guarded tail
    s.template block<true, true>(0);
    int k0 = S::PER;
    for (; k0 + S::PER + S::PD <= s.full_rows; k0 += S::PER) s.template block<false, false>(k0);
    for (; k0 < s.nrows; k0 += S::PER) s.template block<false, true>(k0);
    if (a.detect) s.gate.finish(lane, s.Ti, a.n_ev + b);
}

template <int E, int MR, int NA>
int launch_stream(const AaFastArgs& a, hipStream_t st) {
    const bool det_only = a.detect && !a.P && !a.R && !a.M && !a.valid;
    constexpr int WGD = stream_wg(NA, true), WGS = stream_wg(NA, false);
    const int64_t grid = det_only ? (a.B + WGD / 64 - 1) / (WGD / 64) : (a.B + WGS / 64 - 1) / (WGS / 64);
    // occupancy cap of the two-antenna storing kernel: 24 KiB of LDS per workgroup in all (unused
    // dynamic LDS on top of its 8 KiB lag ring at L 512) = 6 workgroups per CU.  Paired on the
    // reference's detector shape (16384 x 2 x 5315, L 512; 3 rounds, profiles/r06g_occupancy_sweeps.txt):
    // lag ring alone 0.6005 ms, + 8 KiB 0.5843, + 12 KiB 0.5783, + 16 KiB 0.5737, + 20 KiB 0.6044
    // (~27 KiB per workgroup rounds up past 160 KiB / 6: 5 per CU); one antenna at T = 4096 is faster
    // uncapped (1.186 vs 1.228 ms).  variant OCC_LDS (bytes added) overrides.
    using S = AaStream<E, MR, NA, false>;
    constexpr size_t lag_lds = (size_t)(WGS / 64) * (S::LDSLAG ? MR : 1) * NA * S::V4 * 64 * 16;
    constexpr size_t cap_total = 24 * 1024;
    const size_t dflt = (!det_only && NA == 2 && cap_total > lag_lds) ? cap_total - lag_lds : 0;
    const size_t shm = ofs::variant(ofs::V_OCC_LDS) == INT64_MIN ? dflt : ofs::occ_lds();
    if (det_only)
        hipLaunchKernelGGL((aa_stream_kernel<E, MR, NA, true>), dim3((unsigned)grid), dim3(WGD), shm, st, a);
    else
        hipLaunchKernelGGL((aa_stream_kernel<E, MR, NA, false>), dim3((unsigned)grid), dim3(WGS), shm, st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

template <int E, int NA>
int launch_stream_mr(int mr, const AaFastArgs& a, hipStream_t st) {
    switch (mr) {
        case 1: return launch_stream<E, 1, NA>(a, st);
        case 2: return launch_stream<E, 2, NA>(a, st);
        case 4: return launch_stream<E, 4, NA>(a, st);
        case 8: return launch_stream<E, 8, NA>(a, st);
    }
    return 0;
}

// row-scan precision of the register-staged kernel: the detect-only launch scans in fp32, the
// storing launch in fp64; variants FAST_SCAN_DO / FAST_SCAN = 32 | 64 override (tests run the
// storing kernel with the detect-only arithmetic to classify its events, A/B)
bool scan32(bool det_only) {
    const int64_t v = ofs::variant(det_only ? ofs::V_FAST_SCAN_DO : ofs::V_FAST_SCAN);
    if (v == 32 || v == 64) return v == 32;
    return det_only;
}

template <int E, int MR, int NA>
int launch(const AaFastArgs& a, hipStream_t st) {
    const bool det_only = a.detect && !a.P && !a.R && !a.M && !a.valid;
    const bool s32 = scan32(det_only);
    const dim3 grid((unsigned)((a.B + FAST_WG / 64 - 1) / (FAST_WG / 64))), blk(FAST_WG);
    // Occupancy cap: the P/R/M-storing one-antenna kernel runs 10 workgroups (waves) per CU instead
    // of the 12 its 139 VGPRs allow, through 16 KiB of unused dynamic LDS per workgroup (160 KiB per
    // CU / 10).  Paired, 11 rotated rounds on the headline (profiles/r06d_headline_occupancy_sweep.json):
    // 12 per CU 0.2980 ms, 11 0.2920, 10 0.2908, 9 0.2948, 8 0.2954 - fewer streams in flight per CU
    // beat more (so do 3 vs 4 vs 5 waves/SIMD, r06b).  variant FAST_LDS = bytes per workgroup
    // overrides (1: no cap, A/B).
    const int64_t pad = ofs::variant_or(ofs::V_FAST_LDS, (!det_only && NA == 1) ? FAST_CAP_LDS : 0);
    const size_t shm = pad > 0 && pad <= 65536 ? (size_t)pad : 0;
    if (det_only && s32) hipLaunchKernelGGL((aa_fast_kernel<E, MR, NA, true, true>), grid, blk, shm, st, a);
    else if (det_only) hipLaunchKernelGGL((aa_fast_kernel<E, MR, NA, true, false>), grid, blk, shm, st, a);
    else if (s32) hipLaunchKernelGGL((aa_fast_kernel<E, MR, NA, false, true>), grid, blk, shm, st, a);
    else hipLaunchKernelGGL((aa_fast_kernel<E, MR, NA, false, false>), grid, blk, shm, st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

template <int E, int NA, int MR = 1>
int launch_mr(int mr, const AaFastArgs& a, hipStream_t st) {
    if constexpr (MR > TMAX / (64 * E)) {
        return 0;
    } else {
        if (mr == MR) return launch<E, MR, NA>(a, st);
        return launch_mr<E, NA, MR + 1>(mr, a, st);
    }
}

template <int NA>
int launch_e(int E, int mr, const AaFastArgs& a, hipStream_t st) {
    switch (E) {
        case 2: return launch_mr<2, NA>(mr, a, st);
        case 4: return launch_mr<4, NA>(mr, a, st);
        case 8: return launch_mr<8, NA>(mr, a, st);
    }
    return 0;
}

int pick_e(int L) {
    // samples per lane per row; variant FAST_E = 2|4|8 overrides (A/B, parity classification)
    const int forced = (int)ofs::variant_or(ofs::V_FAST_E, 0);
    if (forced == 2 || forced == 4 || forced == 8) return (L % (64 * forced) == 0) ? forced : 0;
    for (int e : {2, 4, 8})                                  // E=2 measured 3 % faster than 4 (r01c)
        if (L % (64 * e) == 0) return e;
    return 0;
}

// detect-only (events without P/R/M stores: VALU/issue-bound, not HBM-bound, SQ counters r03a):
// samples per lane per row.  With fp32 row scans (3 x ~7 VALU per row instead of ~25) E = 4 is
// the fastest (r03f: 0.1071 ms vs 0.1134 at E = 8, 0.1191 / 0.1193 with fp64 scans at E = 4 / 8);
// variant FAST_E_DO = 2|4|8 overrides.
int pick_e_do(int L) {
    const int forced = (int)ofs::variant_or(ofs::V_FAST_E_DO, 0);
    for (int e : {forced, 4, 8, 2})
        if ((e == 2 || e == 4 || e == 8) && L % (64 * e) == 0) return e;
    return 0;
}

}  // namespace

// 10*E + MR of the register-staged kernel (even T <= 1024), 100 + 10*E + MR of the streaming
// kernel (any other T), 0 if the general engine handles the shape
int ofs_aa_fast_plan(int fmt, int precision, int n_ant, int64_t T, int L) {
    if (fmt != OFS_C64 || precision != OFS_FP32) return 0;
    if (n_ant != 1 && n_ant != 2) return 0;
    if (T < 1 || L < 128) return 0;
    if (T <= TMAX && !(T & 1) && L <= TMAX) {
        const int E = pick_e(L);
        if (E) return 10 * E + L / (64 * E);
    }
    if (T > 0x7fffffff - 1024) return 0;                     // row indices in int
    for (int e : {2, 4}) {                                   // streaming: window of 1, 2, 4 or 8 rows
        if (L % (64 * e)) continue;
        const int mr = L / (64 * e);
        if (mr == 1 || mr == 2 || mr == 4 || mr == 8) return 100 + 10 * e + mr;
    }
    return 0;
}

int ofs_aa_fast_try(int fmt, int precision, int n_ant, const AaFastArgs& a, hipStream_t st) {
    const int plan = ofs_aa_fast_plan(fmt, precision, n_ant, a.T, a.L);
    if (!plan) return 0;
    if (plan >= 100) {
        const int E = (plan - 100) / 10, mr = plan % 10;
        if (E == 2) return n_ant == 1 ? launch_stream_mr<2, 1>(mr, a, st) : launch_stream_mr<2, 2>(mr, a, st);
        return n_ant == 1 ? launch_stream_mr<4, 1>(mr, a, st) : launch_stream_mr<4, 2>(mr, a, st);
    }
    int E = plan / 10, mr = plan % 10;
    if (a.detect && !a.P && !a.R && !a.M && !a.valid) {
        // detect-only: its own row width (fewer fp64 row scans per sample); the events are those of
        // the same window sums in another fp32 summation order (parity: oracle/parity.py criterion)
        const int ed = pick_e_do(a.L);
        if (ed) { E = ed; mr = a.L / (64 * ed); }
    }
    return n_ant == 1 ? launch_e<1>(E, mr, a, st) : launch_e<2>(E, mr, a, st);
}
