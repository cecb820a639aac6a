// zc_cfar.hip — zc_v2 CFAR + gate (zc_v2.py:300-346 + :374-446), fused, lane-per-stream recursion.
//
// The only sequential part of zc_streaming_detection is the reference's running sum
// (RunningSum.step, zc_v2.py:219-238): acc = (acc + c[i]) - c[i-W] in float64, left to right.
// Its rounding does not commute, so it is evaluated exactly in that order — but by ONE LANE PER
// STREAM: a workgroup owns ZS streams (16 on the LDS-DMA path), and ZS lanes of its wave 0 (the
// walker) advance the ZS recursions together, one sample per step (2 dependent v_add_f64).
// Everything else is parallel over samples and runs in the ZH helper waves of the workgroup (7 on
// the LDS-DMA path), one chunk behind the walker:
// the threshold flags (corr_scaled >= thresh_scaled, |c| >= min), the stores of every state
// array (coalesced 64-sample rows), and the gate machine in closed form.
//
// Chunks of ZC = 64·ZR samples, staged through LDS (global -> registers -> LDS, two chunks ahead):
//   c tiles (3 buffers: walker reads chunk q while the helpers read chunk q-1 and chunk q+1 lands),
//   c[i-W] tiles (2 buffers, walker only), running-sum tiles (2 buffers, walker -> helpers).
// One barrier per chunk.
//
// Gate (zc_v2.py:374-446) in closed form over the valid samples (valid = i >= W is a prefix):
// with Hp = max(H, 1) and prev(n) the last above sample < n, an open gate closes at the first
// non-above n with n - prev(n) = Hp (the low counter reaches H - 1 before it), and an above
// sample opens a gate iff it is the first one or its gap to prev exceeds Hp (the previous gate
// has closed).  For Hp >= 64 (one row) a row holds at most one close (the carried gate's, at
// prev + Hp, before any above sample of the row) and then at most one open (its first above
// sample).  The peak is the first maximum of c over [gate_start, gate_end] (strict >, the
// opening sample first); gate_mask marks (gate_start, gate_end], and [gate_start, n) for a gate
// still open at the end.  Shorter hysteresis runs the sequential kernel of corr.hip.
#include "ofs_common.h"
#include "ofdmsync.h"

using namespace ofs;

namespace {

// streams per workgroup (walker lanes) and helper waves: LDS-DMA path 16 streams, 11 helpers (one
// workgroup of 12 waves per CU, 154 VGPRs = 3 waves/SIMD; round 5, paired builds on zc_detect: 7 / 8 /
// 11 / 15 helpers 0.306 / 0.289 / 0.286 / 0.492 ms, profiles/r05p_zc_cfar_helpers_ab.txt; static LDS (4 + 3 + 2) x 16 x 130 doubles = 149,760 B = 146.25 KiB of
// gfx950's 160 KiB, asserted in the kernel); register path 8 streams, 3 helpers ((3 + 2 + 2) x 8 x
// 130 doubles = 57 KiB; its staging registers scale with the stream count)
#ifndef OFS_ZC_S
#define OFS_ZC_S 16
#endif
#ifndef OFS_ZC_H
#define OFS_ZC_H 11
#endif
#ifndef OFS_ZC_S_REG
#define OFS_ZC_S_REG 8
#endif
#ifndef OFS_ZC_H_REG
#define OFS_ZC_H_REG 3
#endif
#ifndef OFS_ZC_R
#define OFS_ZC_R 2
#endif
// diagnostic builds: OFS_ZC_NOWALK / OFS_ZC_NOHELP skip the walker / the helpers (timing only)
#ifndef OFS_ZC_NOWALK
#define OFS_ZC_NOWALK 0
#endif
#ifndef OFS_ZC_NOCHAIN
#define OFS_ZC_NOCHAIN 0
#endif
#ifndef OFS_ZC_NOHELP
#define OFS_ZC_NOHELP 0
#endif
constexpr int ZR = OFS_ZC_R;      // 64-sample rows of the gate machine per chunk
constexpr int ZC = 64 * ZR;       // samples per chunk
constexpr int ZP = ZC + 2;        // LDS row pitch in doubles (16-byte rows; walker column reads spread over banks)

struct ZcArgs {
    const double* mag;
    int64_t B, n;
    int W; double tv, scale, minmag; int reflen, Hp;
    double* local_sum; double* corr_scaled; double* thresh_scaled;
    uint8_t* above; uint8_t* valid; uint8_t* gate_mask;
    int max_ev; int32_t* n_ev; int64_t* ev; double* ev_v;
};

// per-stream gate state, wave-uniform in the helper wave that owns the stream
struct ZGate {
    int64_t last_above;     // last above sample (< current row), -1 if none
    int64_t gs, pk;
    double pv;
    int open, nev;
};

// DMA: the walker stages the c / c[i-W] tiles with LDS-DMA (global_load_lds_dwordx4, no
// registers), two chunks ahead of use instead of one (the register path's loads land one chunk
// period after they are issued, so a chunk could not be shorter than a memory round trip);
// taken when every tile row is a whole, 16-byte-aligned 1 KiB span (host checks).

#ifndef OFS_ZC_TIMING
#define OFS_ZC_TIMING 0            // diagnostic builds: per-role cycles (tools/zc_phase.py)
#endif
#if OFS_ZC_TIMING
__device__ unsigned long long zc_prof[8];
__device__ unsigned zc_hwid[4096 * 8];       // HW_ID of every wave (workgroup-major), first launch rows
#define ZC_T(i)                                                                                      \
    if (lane == 0) { const long long t_ = __builtin_amdgcn_s_memtime(); tacc[i] += t_ - tprev; tprev = t_; }
#else
#define ZC_T(i)
#endif
#ifndef OFS_ZC_ZB
#define OFS_ZC_ZB 8                // walker: samples per LDS batch (read one batch ahead of the adds)
#endif
#ifndef OFS_ZC_DIAG_NOLDS
#define OFS_ZC_DIAG_NOLDS 0        // diagnostic builds (timing only, wrong results): helpers read no LDS
#endif
#ifndef OFS_ZC_DIAG_NOST
#define OFS_ZC_DIAG_NOST 0         // ... helpers store nothing on quiet chunks
#endif
#ifndef OFS_ZC_WUNROLL
#define OFS_ZC_WUNROLL 16          // walker: LDS batches unrolled per chunk (code size A/B)
#endif
#ifndef OFS_ZC_HUNROLL
#define OFS_ZC_HUNROLL 2           // helpers: rows of the gate pass unrolled (code size A/B)
#endif
#ifndef OFS_ZC_ISOLATE
#define OFS_ZC_ISOLATE 0           // 1: the walker's SIMD-mates idle (A/B, r05ao: bit-identical, 0.2925 vs
                                   // 0.2864 ms with 9 working helpers; 13 waves 0.444 - SIMD sharing is
                                   // not what slows the walker's chain, as round 3 found by other means)
#endif
#ifndef OFS_ZC_QUIET
#define OFS_ZC_QUIET 1             // 0: gate machine on every row (A/B)
#endif
// state / mask stores of the helpers: non-temporal (streamed past the caches; nothing here reads
// them back).  r05av, bit-identical: state arrays 0.63 -> 0.56 ms, events + mask unchanged (0.286)
#ifndef OFS_ZC_NT
#define OFS_ZC_NT 1
#endif
// helpers read c from global memory (L2: the walker's DMA brought the rows in) instead of the LDS
// tile, template HG: taken when state arrays are stored (paired, r06k: state mode 0.564 -> 0.540 ms;
// events + mask only 0.285 -> 0.342 ms, so not there); OFS_ZC_HGLOBAL = 1 forces it (A/B)
#ifndef OFS_ZC_HGLOBAL
#define OFS_ZC_HGLOBAL 0
#endif
template <class T>
__device__ __forceinline__ void zc_st(T* p, T v) {
#if OFS_ZC_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// walker: the exact left-to-right recursion of RunningSum.step over one full chunk of this lane's
// stream; LDS reads a batch ahead of the dependent adds (the chain is 2 v_add_f64 per sample; an
// LDS round trip per sample would set the pace instead).  OZ: c[i-W] is 0 (window not yet full).
template <int ZCN, bool OZ>
__device__ __forceinline__ void zc_walk_chunk(const double* x, const double* o, double* r, double& acc) {
#pragma clang fp contract(off)
    constexpr int ZB = OFS_ZC_ZB;
    double2 xv[ZB / 2], ov[ZB / 2];
#pragma unroll
    for (int j = 0; j < ZB / 2; ++j) {
        xv[j] = reinterpret_cast<const double2*>(x)[j];
        if (!OZ) ov[j] = reinterpret_cast<const double2*>(o)[j];
    }
#pragma unroll OFS_ZC_WUNROLL
    for (int bb = 0; bb < ZCN / ZB; ++bb) {
        double2 xn[ZB / 2], on[ZB / 2];
        if (bb + 1 < ZCN / ZB) {
#pragma unroll
            for (int j = 0; j < ZB / 2; ++j) {
                xn[j] = reinterpret_cast<const double2*>(x + (bb + 1) * ZB)[j];
                if (!OZ) on[j] = reinterpret_cast<const double2*>(o + (bb + 1) * ZB)[j];
            }
        }
#pragma unroll
        for (int j = 0; j < ZB / 2; ++j) {
            double2 rr;
#if OFS_ZC_NOCHAIN
            rr.x = xv[j].x - (OZ ? 0.0 : ov[j].x); rr.y = xv[j].y - (OZ ? 0.0 : ov[j].y);
#else
            if (OZ) {
                acc = acc + xv[j].x; rr.x = acc;
                acc = acc + xv[j].y; rr.y = acc;
            } else {
                acc = (acc + xv[j].x) - ov[j].x; rr.x = acc;
                acc = (acc + xv[j].y) - ov[j].y; rr.y = acc;
            }
#endif
            reinterpret_cast<double2*>(r + bb * ZB)[j] = rr;
        }
        if (bb + 1 < ZCN / ZB) {
#pragma unroll
            for (int j = 0; j < ZB / 2; ++j) { xv[j] = xn[j]; if (!OZ) ov[j] = on[j]; }
        }
    }
}

template <bool DMA, int ZS, int ZH, bool HG>
__global__ __launch_bounds__(64 * (1 + ZH))
void zc_cfar_kernel(ZcArgs a) {
#pragma clang fp contract(off)
#if OFS_ZC_TIMING
    long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long tprev = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096 && threadIdx.x / 64 < 8)
        zc_hwid[blockIdx.x * 8 + threadIdx.x / 64] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
#endif
    constexpr int NC = DMA ? 4 : 3, NO = DMA ? 3 : 2;
    constexpr int ZDMA_PER_CHUNK = 2 * ZS * (ZC / 128);   // DMA instructions per chunk (c and c[i-W])
    __shared__ double tc[NC][ZS][ZP];     // c
    __shared__ double to[NO][ZS][ZP];     // c[i - W] (0 before the window fills)
    __shared__ double ta[2][ZS][ZP];      // running sum after sample i
    static_assert(sizeof(tc) + sizeof(to) + sizeof(ta) <= 160 * 1024,
                  "zc_cfar_kernel: static LDS beyond gfx950's 160 KiB per workgroup (OFS_ZC_S / ZC / ZP)");
    const int lane = threadIdx.x & 63;
    // role of this wave: 0 = walker, 1..ZH = helpers.  (Measured and not kept: the walker chosen by
    // SIMD id so both workgroups' walkers share a SIMD, 0.38 -> 0.45 ms; an idle 8th wave as the
    // walker's SIMD partner, 0.362 -> 0.373 ms: SIMD sharing is not what slows the chain.)
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    // OFS_ZC_ISOLATE: a workgroup's waves go to the CU's SIMDs in a fixed cyclic order (wave w shares
    // the SIMD of wave w mod 4), so waves 4, 8, ... would share the walker's SIMD and take issue
    // slots from its dependent chain; they idle (barriers only) and the other waves are the helpers
    constexpr int ZHE = OFS_ZC_ISOLATE ? ZH - ZH / 4 : ZH;            // helper waves doing work
    constexpr int NJ = (ZS + ZHE - 1) / ZHE;                         // streams per helper wave
    const bool idle_w = OFS_ZC_ISOLATE && wv > 0 && (wv & 3) == 0;
    const int hi = OFS_ZC_ISOLATE ? wv - 1 - (wv >> 2) : wv - 1;     // helper rank (valid if !idle_w)
    const int64_t b0 = (int64_t)blockIdx.x * ZS;
    const int ns = (int)min((int64_t)ZS, a.B - b0);          // streams of this workgroup
    const int64_t n = a.n;
    const int nch = (int)((n + ZC - 1) / ZC);

    // loader = the walker wave, which issues no global stores: its wait for the loads of the next
    // chunk (staged one iteration after they are issued) never drains the helpers' stores
    // loader = the walker wave, which issues no global stores: its wait for the loads of the next
    // chunk (staged one iteration after they are issued) never drains the helpers' stores.
    // (Two register sets, loads two chunks ahead: measured slower, 0.64 vs 0.46 ms.)
    double pc[ZR][ZS], po[ZR][ZS];
    const double* cw = a.mag + b0 * n;                        // this workgroup's streams
    auto load = [&](int q) {
#pragma unroll
        for (int rr = 0; rr < ZR; ++rr) {
            const int64_t i = (int64_t)q * ZC + 64 * rr + lane;
#pragma unroll
            for (int s = 0; s < ZS; ++s) {
                const bool ok = s < ns && i < n;
                pc[rr][s] = ok ? cw[s * n + i] : 0.0;
                po[rr][s] = (ok && i >= a.W) ? cw[s * n + i - a.W] : 0.0;
            }
        }
    };
    auto stage = [&](int q) {
#pragma unroll
        for (int rr = 0; rr < ZR; ++rr)
#pragma unroll
            for (int s = 0; s < ZS; ++s) {
                tc[q % NC][s][64 * rr + lane] = pc[rr][s];
                to[q % NO][s][64 * rr + lane] = po[rr][s];
            }
    };
    // DMA path: 1 KiB per instruction (64 lanes x 16 B); rows of absent streams re-read the last
    // stream (unused); c[i-W] tiles of chunks before the window fills copy the c tile (the walker
    // uses zeros there: W is a whole number of chunks on this path)
    auto dma = [&](int q) {
#pragma unroll
        for (int s = 0; s < ZS; ++s) {
            const int ss = s < ns ? s : ns - 1;
            const double* src = cw + (int64_t)ss * n + (int64_t)q * ZC + 2 * lane;
            const double* srco = (int64_t)q * ZC >= a.W ? src - a.W : src;
#pragma unroll
            for (int j = 0; j < ZC / 128; ++j) {
                lds_dma16(src + 128 * j, &tc[q % NC][s][128 * j]);
                lds_dma16(srco + 128 * j, &to[q % NO][s][128 * j]);
            }
        }
    };

    ZGate g[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { g[j].last_above = -1; g[j].gs = 0; g[j].pk = 0; g[j].pv = 0.0; g[j].open = 0; g[j].nev = 0; }
    double acc = 0.0;                                         // walker lane s < ns: stream b0 + s

    // LDS-only barrier: the helpers' global stores are never waited for (a __syncthreads() fence
    // would drain them, a full store round trip per chunk); the loads are staged one iteration
    // after they are issued, so their wait overlaps a whole chunk of work
    auto lds_barrier = [] {
        if constexpr (DMA) {
            // no memory-model fence here: with LDS-DMA in the kernel the compiler implements a
            // "local" release fence as vmcnt(0), which would drain the DMAs in flight (and the
            // helpers' stores) every chunk.  This wave's LDS accesses complete at lgkmcnt(0); the
            // DMA'd tiles a chunk reads were waited for by the walker before the barrier.
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        }
    };
    if (wv == 0) {
        if constexpr (DMA) {
            dma(0);
            if (1 < nch) dma(1);
        } else {
            load(0);
            stage(0);
            if (1 < nch) load(1);
        }
    }
    lds_barrier();
    for (int q = 0; q <= nch; ++q) {
        if (wv == 0) {
            if constexpr (DMA) {
                if (q + 2 < nch) dma(q + 2);
                // chunk q has landed once at most the (up to two) later chunks' DMAs are in flight
                // (loads complete in order, so "at most min(63, later x per-chunk) outstanding"
                // implies chunk q has landed; 63 = the vmcnt field's maximum)
                constexpr int V2 = 2 * ZDMA_PER_CHUNK < 63 ? 2 * ZDMA_PER_CHUNK : 63;
                constexpr int V1 = ZDMA_PER_CHUNK < 63 ? ZDMA_PER_CHUNK : 63;
                const int later = min(2, nch - 1 - q);
                if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(V2) : "memory");
                else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(V1) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                ZC_T(0)
            } else {
                if (q + 1 < nch) stage(q + 1);                // loaded during the previous chunk
                if (q + 2 < nch) load(q + 2);
            }
        }
        if (wv == 0) {
            // ---- walker: the exact left-to-right recursion of RunningSum.step ----
            if (!OFS_ZC_NOWALK && q < nch && lane < ZS) {
                const int cnt = (int)min((int64_t)ZC, n - (int64_t)q * ZC);
                const double* x = tc[q % NC][lane];
                const double* o = to[q % NO][lane];
                const bool ozero = DMA && (int64_t)q * ZC < a.W;      // DMA path: before the window fills
                double* r = ta[q & 1][lane];
                if (cnt == ZC) {
                    // ozero is uniform per chunk: a chain without the c[i-W] reads and selects
                    // (x - 0.0 == x exactly, -0.0 included) instead of two v_cndmask per sample
                    if (ozero) zc_walk_chunk<ZC, true>(x, o, r, acc);
                    else zc_walk_chunk<ZC, false>(x, o, r, acc);
                } else {
                    for (int u = 0; u < cnt; ++u) { acc = (acc + x[u]) - (ozero ? 0.0 : o[u]); r[u] = acc; }
                }
            }
            ZC_T(1)
        } else if (!OFS_ZC_NOHELP && q >= 1 && !idle_w) {
            // ---- helpers: chunk q-1 (flags, stores, gate) ----
            const int qc = q - 1;
            // pass 1 (OFS_ZC_QUIET): the flags of every (row, stream) of this wave.  A chunk with no
            // above sample and no open gate (the common case: events are sparse) needs no gate
            // logic - its gate_mask rows are 0 - so the wave skips the scalar gate machine.
            bool quiet = OFS_ZC_QUIET != 0;
            double cv[ZR][NJ], lv[ZR][NJ];
            uint64_t am[ZR][NJ];
            // every LDS read of the chunk first (one latency for all of them, not one per row),
            // then the flags with non-short-circuit logic (no exec-mask branches per term)
#pragma unroll
            for (int rr = 0; rr < ZR; ++rr)
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int s = hi + ZHE * j;
                    const int sr = s < ns ? s : 0;
#if OFS_ZC_DIAG_NOLDS                                           // diagnostic: no helper LDS reads
                    cv[rr][j] = 1e-3 * (double)(lane + sr) + (double)qc; lv[rr][j] = cv[rr][j] * 1e30;
#else
                    if constexpr (HG || OFS_ZC_HGLOBAL) {
                        const int64_t ig = (int64_t)qc * ZC + 64 * rr + lane;
                        cv[rr][j] = ig < n ? cw[(int64_t)sr * n + ig] : 0.0;
                    } else {
                        cv[rr][j] = tc[qc % NC][sr][64 * rr + lane];
                    }
                    lv[rr][j] = ta[qc & 1][sr][64 * rr + lane];
#endif
                }
#pragma unroll
            for (int rr = 0; rr < ZR; ++rr) {
                const int64_t i = (int64_t)qc * ZC + 64 * rr + lane;
                const bool vd = (i < n) & (i >= a.W);
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int s = hi + ZHE * j;
                    const bool ab = (s < ns) & vd & (cv[rr][j] * a.scale >= lv[rr][j] * a.tv) & (cv[rr][j] >= a.minmag);
                    am[rr][j] = __ballot(ab);
                    if (am[rr][j]) quiet = false;
                }
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                if (g[j].open) quiet = false;
#pragma unroll OFS_ZC_HUNROLL
            for (int rr = 0; rr < ZR; ++rr) {
            const int64_t base = (int64_t)qc * ZC + 64 * rr;
            const int64_t i = base + lane;
            const bool inb = i < n;
            const bool vd = inb && i >= a.W;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int s = hi + ZHE * j;
                if (s >= ns) break;
                const double c = cv[rr][j];
                const double ls = lv[rr][j];
                const double cs = c * a.scale, th = ls * a.tv;
                const uint64_t abm = am[rr][j];
                const bool ab = (abm >> lane) & 1;
                const int64_t o = (b0 + s) * n + i;
                if (quiet) {
                    if (inb && !OFS_ZC_DIAG_NOST) {
                        if (a.local_sum) zc_st(&a.local_sum[o], ls);
                        if (a.corr_scaled) zc_st(&a.corr_scaled[o], cs);
                        if (a.thresh_scaled) zc_st(&a.thresh_scaled[o], th);
                        if (a.above) zc_st(&a.above[o], (uint8_t)0);
                        if (a.valid) zc_st(&a.valid[o], (uint8_t)vd);
                        if (a.gate_mask) zc_st(&a.gate_mask[o], (uint8_t)0);
                    }
                    continue;
                }
                ZGate& G = g[j];
                // gate in closed form (Hp >= 64): carried close first, then this row's first above
                int close_l = -1;                                     // row lane of the close
                if (G.open) {
                    const int64_t nc = G.last_above + a.Hp;
                    const int64_t fa = abm ? base + __builtin_ctzll(abm) : INT64_MAX;
                    if (nc >= base && nc < base + 64 && nc < n && fa > nc) close_l = (int)(nc - base);
                }
                const int open_l = abm ? __builtin_ctzll(abm) : -1;
                const bool carried = G.open != 0;
                const bool opens = open_l >= 0 && (!carried || close_l >= 0);   // Hp >= 64: open after close
                // gate_mask: carried gate over [0, close] (or the whole row), new gate over (open, 63]
                const int cend = carried ? (close_l >= 0 ? close_l : 63) : -1;
                const bool mk = inb && ((lane <= cend) || (opens && lane > open_l));
                if (carried) {                                       // peak over [0, cend]
                    const double v = (inb && lane <= cend) ? c : -__builtin_huge_val();
                    const double m = wave_max(v);
                    if (m > G.pv) {
                        const uint64_t at = __ballot(inb && lane <= cend && c == m);
                        G.pv = m; G.pk = base + __builtin_ctzll(at);
                    }
                    if (close_l >= 0) {
                        if (a.ev && G.nev < a.max_ev && lane < 4) {
                            int64_t* r = a.ev + ((b0 + s) * (int64_t)a.max_ev + G.nev) * 4;
                            const int64_t ds = G.pk - a.reflen + 1 > 0 ? G.pk - a.reflen + 1 : 0;
                            r[lane] = lane == 0 ? G.pk : lane == 1 ? G.gs : lane == 2 ? base + close_l : ds;
                            if (lane == 0 && a.ev_v) a.ev_v[(b0 + s) * (int64_t)a.max_ev + G.nev] = G.pv;
                        }
                        G.nev += 1; G.open = 0; G.pv = 0.0;
                    }
                }
                if (opens) {                                         // opening sample, then (open, 63]
                    G.open = 1; G.gs = base + open_l; G.pk = G.gs;
                    G.pv = readlane(c, open_l);
                    const double v = (inb && lane > open_l) ? c : -__builtin_huge_val();
                    const double m = wave_max(v);
                    if (m > G.pv) {
                        const uint64_t at = __ballot(inb && lane > open_l && c == m);
                        G.pv = m; G.pk = base + __builtin_ctzll(at);
                    }
                }
                if (abm) G.last_above = base + 63 - __builtin_clzll(abm);
                if (inb) {
                    if (a.local_sum) zc_st(&a.local_sum[o], ls);
                    if (a.corr_scaled) zc_st(&a.corr_scaled[o], cs);
                    if (a.thresh_scaled) zc_st(&a.thresh_scaled[o], th);
                    if (a.above) zc_st(&a.above[o], (uint8_t)ab);
                    if (a.valid) zc_st(&a.valid[o], (uint8_t)vd);
                    if (a.gate_mask) zc_st(&a.gate_mask[o], (uint8_t)mk);
                }
            }
            }
            ZC_T(3)
        }
        lds_barrier();
        if (wv == 0) { ZC_T(2) } else { ZC_T(4) }
    }
    // ---- gates still open at the end: gate_end = n, gate_mask[gate_start:n] ----
    if (wv >= 1 && !idle_w) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int s = hi + ZHE * j;
            if (s >= ns) break;
            ZGate& G = g[j];
            if (G.open) {
                if (a.ev && G.nev < a.max_ev && lane < 4) {
                    int64_t* r = a.ev + ((b0 + s) * (int64_t)a.max_ev + G.nev) * 4;
                    const int64_t ds = G.pk - a.reflen + 1 > 0 ? G.pk - a.reflen + 1 : 0;
                    r[lane] = lane == 0 ? G.pk : lane == 1 ? G.gs : lane == 2 ? n : ds;
                    if (lane == 0 && a.ev_v) a.ev_v[(b0 + s) * (int64_t)a.max_ev + G.nev] = G.pv;
                }
                G.nev += 1;
                if (lane == 0 && a.gate_mask) a.gate_mask[(b0 + s) * n + G.gs] = 1;
            }
            if (lane == 0 && a.n_ev) a.n_ev[b0 + s] = G.nev;
        }
    }
#if OFS_ZC_TIMING
    if (lane == 0)
        for (int i = 0; i < 5; ++i) atomicAdd(&zc_prof[i], (unsigned long long)tacc[i]);
#endif
}

}  // namespace

// fused CFAR + gate for hysteresis >= one chunk; returns 0 when the shape is not covered
int ofs_zc_cfar_try(const double* corr_mag, int64_t B, int64_t n, int W, double tv, double scale,
                    double minmag, int reflen, int hyst, double* local_sum, double* corr_scaled,
                    double* thresh_scaled, uint8_t* above, uint8_t* valid, uint8_t* gate_mask, int max_ev,
                    int32_t* n_ev, int64_t* ev, double* ev_v, hipStream_t st) {
    const int Hp = hyst > 1 ? hyst : 1;
    if (Hp < 64 || B <= 0 || n <= 0 || ofs::variant_on(ofs::V_ZC_SEQ)) return 0;
    ZcArgs a{corr_mag, B, n, W, tv, scale, minmag, reflen, Hp, local_sum, corr_scaled, thresh_scaled,
             above, valid, gate_mask, max_ev, n_ev, ev, ev_v};
    constexpr int SD = OFS_ZC_S, HD = OFS_ZC_H, SR = OFS_ZC_S_REG, HR = OFS_ZC_H_REG;
    const bool dma = ZC % 128 == 0 && n % ZC == 0 && W % ZC == 0 && W >= 0 &&
                     (reinterpret_cast<uintptr_t>(corr_mag) & 15) == 0 && !ofs::variant_on(ofs::V_ZC_NODMA);
    const bool state = local_sum || corr_scaled || thresh_scaled;
    const dim3 gd((unsigned)((B + SD - 1) / SD)), gr((unsigned)((B + SR - 1) / SR));
    if (dma && state) hipLaunchKernelGGL((zc_cfar_kernel<true, SD, HD, true>), gd, dim3(64 * (1 + HD)), 0, st, a);
    else if (dma) hipLaunchKernelGGL((zc_cfar_kernel<true, SD, HD, false>), gd, dim3(64 * (1 + HD)), 0, st, a);
    else hipLaunchKernelGGL((zc_cfar_kernel<false, SR, HR, false>), gr, dim3(64 * (1 + HR)), 0, st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

#if OFS_ZC_TIMING
// per-role cycle totals of zc_cfar_kernel since the last call (diagnostic builds): walker DMA wait,
// walker chain, walker barrier, helper work, helper barrier
extern "C" int ofs_zc_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(zc_prof), 5 * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(zc_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
extern "C" int ofs_zc_hwid(unsigned* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(zc_hwid), 4096 * 8 * sizeof(unsigned)) == hipSuccess ? 0 : -1;
}
#endif
