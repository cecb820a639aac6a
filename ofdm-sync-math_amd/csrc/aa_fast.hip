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
// (ofdmsync.hip), streamed row by row: prev-above by lane-serial + DPP max-scan,
// opens/closes by ballot, per-gate argmax by wave reductions, scalar carry between rows.
#include "ofs_common.h"
#include "ofdmsync.h"

using namespace ofs;

namespace {

constexpr int FAST_WG = 256;      // 4 waves = 4 independent streams per workgroup
constexpr int TMAX = 1024;        // stream length handled by the fast path
constexpr int NOKEY = 1 << 20;

// zero-filled DPP move (bound_ctrl): lanes without a source read 0
template <int CTRL, int RMASK = 0xf>
__device__ __forceinline__ double dppz(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, RMASK, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, RMASK, 0xf, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double scan_add(double v) {
    v += dppz<0x111>(v);            // row_shr:1
    v += dppz<0x112>(v);            // row_shr:2
    v += dppz<0x114>(v);            // row_shr:4
    v += dppz<0x118>(v);            // row_shr:8
    v += dppz<0x142, 0xa>(v);       // row_bcast:15 -> rows 1, 3
    v += dppz<0x143, 0xc>(v);       // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ double shr1z(double v) { return dppz<0x138>(v); }   // wave_shr:1, lane 0 <- 0

template <int NA, int E, int MR>
__global__ __launch_bounds__(FAST_WG) void aa_fast_kernel(AaFastArgs a) {
    constexpr int RL = 64 * E;                 // samples per row
    constexpr int RW = TMAX / RL;              // rows per stream
    constexpr int L = MR * RL;
    constexpr int V4 = E / 2;                  // float4 (2 samples) per lane per row
    static_assert(MR >= 1 && MR <= RW, "window must fit the stream tile");
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * (FAST_WG / 64) + (threadIdx.x >> 6);
    if (b >= a.B) return;
    const int T = (int)a.T;
    const float4* xin = reinterpret_cast<const float4*>(a.x);

    // ---- every load of the stream up front: RW x V4 x NA dwordx4 per lane ----
    float4 xv[NA][RW][V4];
#pragma unroll
    for (int k = 0; k < RW; ++k)
#pragma unroll
        for (int j = 0; j < V4; ++j) {
            const int n = RL * k + E * lane + 2 * j;
#pragma unroll
            for (int br = 0; br < NA; ++br)
                xv[br][k][j] = (n < T) ? xin[((b * NA + br) * a.T + n) >> 1] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    auto xat = [&](int br, int k, int e, double& re, double& im) {
        float fr, fi;
        const float4 v = xv[br][k][e >> 1];
        if (e & 1) { fr = v.z; fi = v.w; } else { fr = v.x; fi = v.y; }
        asm volatile("" : "+v"(fr), "+v"(fi));   // keep samples fp32 in registers: convert at use
        re = fr; im = fi;
    };

    float sR[MR][E], sI[MR][E], sE[MR][E];      // retained in-window suffixes (ring by k % MR)
    double Cr[RW + 1], Ci[RW + 1], Ce[RW + 1];  // running row bases (wave-uniform)
    Cr[0] = Ci[0] = Ce[0] = 0.0;

    // event state (wave-uniform)
    const int Hp = a.hyst > 1 ? a.hyst : 1;
    int carry_last = -1, n_ev = 0, ev_start = 0, gate_open = 0, bidx = 0;
    float bpm = -1.f, bpr = 0.f, bpi = 0.f, bm = 0.f;
    int64_t* evi = a.detect ? a.ev_i + b * (int64_t)a.max_ev * 4 : nullptr;
    double* evr = a.detect ? a.ev_r + b * (int64_t)a.max_ev * 4 : nullptr;
    auto emit = [&](int gate_end) {
        if (lane == 0 && n_ev < a.max_ev) {
            int64_t* ei = evi + (int64_t)n_ev * 4;
            double* er = evr + (int64_t)n_ev * 4;
            ei[0] = bidx; ei[1] = ev_start; ei[2] = gate_end; ei[3] = (int64_t)bidx - 2 * L + 1;
            er[0] = bpr; er[1] = bpi; er[2] = bm;
            er[3] = atan2((double)bpi, (double)bpr) * a.fs / (2.0 * M_PI * (double)L);
        }
        n_ev += 1;
    };

    float* Pout = reinterpret_cast<float*>(a.P);
    float* Rout = reinterpret_cast<float*>(a.R);
    float* Mout = reinterpret_cast<float*>(a.M);

#pragma unroll
    for (int k = 0; k < RW; ++k) {
        if (RL * k < T) {                                       // wave-uniform row guard
            const int nb = RL * k + E * lane;                   // first sample of this lane
            // ---- pass 1: lane totals of products / energies, wave scan ----
            double tR = 0.0, tI = 0.0, tE = 0.0;
#pragma unroll
            for (int e = 0; e < E; ++e)
#pragma unroll
                for (int br = 0; br < NA; ++br) {
                    double xr, xi;
                    xat(br, k, e, xr, xi);
                    tE += xr * xr + xi * xi;
                    if (k >= MR) {
                        double dr, di;
                        xat(br, k - MR, e, dr, di);
                        tR += xr * dr + xi * di;                 // x[n]·conj(x[n-L])
                        tI += xi * dr - xr * di;
                    }
                }
            const double iR = scan_add(tR), iI = scan_add(tI), iE = scan_add(tE);
            double rR = shr1z(iR), rI = shr1z(iI), rE = shr1z(iE);   // exclusive in-row prefix
            const double totR = readlane(iR, 63), totI = readlane(iI, 63), totE = readlane(iE, 63);
            Cr[k + 1] = Cr[k] + totR; Ci[k + 1] = Ci[k] + totI; Ce[k + 1] = Ce[k] + totE;
            // rows strictly inside the window (k >= MR) or everything before row k (k < MR)
            const double fR = (k >= MR) ? (Cr[k] - Cr[k - MR + 1]) : Cr[k];
            const double fI = (k >= MR) ? (Ci[k] - Ci[k - MR + 1]) : Ci[k];
            const double fE = (k >= MR) ? (Ce[k] - Ce[k - MR + 1]) : Ce[k];

            // ---- pass 2: recompute products, window sums, metric, outputs ----
            float pf[E][2], mf[E], pmf[E], rf[E], nsR[E], nsI[E], nsE[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                double aR = 0.0, aI = 0.0, aE = 0.0;
#pragma unroll
                for (int br = 0; br < NA; ++br) {
                    double xr, xi;
                    xat(br, k, e, xr, xi);
                    aE += xr * xr + xi * xi;
                    if (k >= MR) {
                        double dr, di;
                        xat(br, k - MR, e, dr, di);
                        aR += xr * dr + xi * di;
                        aI += xi * dr - xr * di;
                    }
                }
                rR += aR; rI += aI; rE += aE;                   // inclusive in-row prefix
                double PR = rR + fR, PI = rI + fI, RR = rE + fE;
                if (k >= MR) {
                    PR += (double)sR[k % MR][e]; PI += (double)sI[k % MR][e]; RR += (double)sE[k % MR][e];
                }
                nsR[e] = (float)(totR - rR); nsI[e] = (float)(totI - rI); nsE[e] = (float)(totE - rE);
                const double pm = PR * PR + PI * PI;
                double m = 0.0;
                if (k >= MR && RR > 1e-6 * (double)L) {
                    m = pm / (RR * RR);
                    m = m < 1.0 ? m : 1.0;
                }
                pf[e][0] = (float)PR; pf[e][1] = (float)PI;
                rf[e] = (float)RR; mf[e] = (float)m; pmf[e] = (float)pm;
            }
#pragma unroll
            for (int e = 0; e < E; ++e) { sR[k % MR][e] = nsR[e]; sI[k % MR][e] = nsI[e]; sE[k % MR][e] = nsE[e]; }

            const int64_t o = b * a.T + nb;
#pragma unroll
            for (int j = 0; j < V4; ++j) {
                if (nb + 2 * j < T) {
                    if (Pout) *reinterpret_cast<float4*>(Pout + 2 * (o + 2 * j)) =
                        make_float4(pf[2 * j][0], pf[2 * j][1], pf[2 * j + 1][0], pf[2 * j + 1][1]);
                    if constexpr (E % 4 != 0) {
                        if (Rout) *reinterpret_cast<float2*>(Rout + o + 2 * j) = make_float2(rf[2 * j], rf[2 * j + 1]);
                        if (Mout) *reinterpret_cast<float2*>(Mout + o + 2 * j) = make_float2(mf[2 * j], mf[2 * j + 1]);
                    } else if ((j & 1) == 0) {
                        if (Rout) *reinterpret_cast<float4*>(Rout + o + 2 * j) =
                            make_float4(rf[2 * j], rf[2 * j + 1], rf[2 * j + 2], rf[2 * j + 3]);
                        if (Mout) *reinterpret_cast<float4*>(Mout + o + 2 * j) =
                            make_float4(mf[2 * j], mf[2 * j + 1], mf[2 * j + 2], mf[2 * j + 3]);
                    }
                    if (a.valid) { a.valid[o + 2 * j] = (k >= MR); a.valid[o + 2 * j + 1] = (k >= MR); }
                }
            }

            // ---- events: closed-form gate machine, streamed per row ----
            if (a.detect && k >= MR) {
                bool ab[E];
                int lane_last = -1;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    ab[e] = (nb + e < T) && (double)mf[e] >= a.thr;
                    if (ab[e]) lane_last = nb + e;
                }
                const int W = max(wave_scan_max(lane_last, lane), carry_last);
                int run = wave_shr1(W, lane, carry_last);
                uint64_t Om[E], Cm[E];
                uint64_t any = 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int n = nb + e;
                    const int pe = run;
                    if (ab[e]) run = n;
                    const bool cl = (n < T) && run >= 0 && (n - run) == Hp;
                    const bool op = ab[e] && (pe < 0 || (n - 1 - pe) >= Hp);
                    Om[e] = __ballot(op);
                    Cm[e] = __ballot(cl);
                    any |= Om[e] | Cm[e];
                }
                carry_last = readlane(W, 63);

                auto seg_reduce = [&](int lo, int hi) {        // first argmax of |P|² on keys [lo, hi]
                    float c[E];
                    float lm = -1.f;
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int key = E * lane + e;
                        c[e] = (nb + e < T && key >= lo && key <= hi) ? pmf[e] : -1.f;
                        lm = fmaxf(lm, c[e]);
                    }
                    const float vmax = wave_max(lm);
                    int kk = NOKEY;
#pragma unroll
                    for (int e = E - 1; e >= 0; --e)
                        if (c[e] == vmax) kk = E * lane + e;
                    kk = wave_min(kk);
                    if (vmax > bpm && kk != NOKEY) {
                        const int ln = kk / E, es = kk % E;
                        float sel_pr = pf[0][0], sel_pi = pf[0][1], sel_m = mf[0];
#pragma unroll
                        for (int e = 1; e < E; ++e)
                            if (es == e) { sel_pr = pf[e][0]; sel_pi = pf[e][1]; sel_m = mf[e]; }
                        bpr = readlane(sel_pr, ln);
                        bpi = readlane(sel_pi, ln);
                        bm = readlane(sel_m, ln);
                        bpm = vmax;
                        bidx = RL * k + kk;
                    }
                };

                int seg_lo = gate_open ? 0 : -1;
                if (any) {
                    int pos = -1;
                    while (true) {
                        int key = NOKEY, is_open = 0;
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int q = pos - e;
                            const int t = q < 0 ? 0 : q / E + 1;       // lanes whose key > pos
                            const uint64_t msk = t >= 64 ? 0ull : (~0ull << t);
                            const uint64_t o = Om[e] & msk, c = Cm[e] & msk;
                            if (o) { const int kq = E * __builtin_ctzll(o) + e; if (kq < key) { key = kq; is_open = 1; } }
                            if (c) { const int kq = E * __builtin_ctzll(c) + e; if (kq < key) { key = kq; is_open = 0; } }
                        }
                        if (key == NOKEY) break;
                        if (is_open) {
                            gate_open = 1; ev_start = RL * k + key; seg_lo = key; bpm = -1.f;
                        } else {
                            seg_reduce(seg_lo, key);
                            emit(RL * k + key);
                            gate_open = 0; seg_lo = -1;
                        }
                        pos = key;
                    }
                }
                if (gate_open) seg_reduce(seg_lo, RL - 1);
            }
        }
    }
    if (a.detect) {
        if (gate_open) emit(T);
        if (lane == 0) a.n_ev[b] = n_ev;
    }
}

template <int NA, int E, int MR>
int launch(const AaFastArgs& a, hipStream_t st) {
    const int64_t grid = (a.B + 3) / 4;
    hipLaunchKernelGGL((aa_fast_kernel<NA, E, MR>), dim3((unsigned)grid), dim3(FAST_WG), 0, st, a);
    return hipGetLastError() == hipSuccess ? 1 : OFS_EHIP;
}

template <int NA, int E, int MR = 1>
int launch_mr(int mr, const AaFastArgs& a, hipStream_t st) {
    if constexpr (MR > TMAX / (64 * E)) {
        return 0;
    } else {
        if (mr == MR) return launch<NA, E, MR>(a, st);
        return launch_mr<NA, E, MR + 1>(mr, a, st);
    }
}

template <int NA>
int launch_e(int E, int mr, const AaFastArgs& a, hipStream_t st) {
    switch (E) {
        case 2: return launch_mr<NA, 2>(mr, a, st);
        case 4: return launch_mr<NA, 4>(mr, a, st);
        case 8: return launch_mr<NA, 8>(mr, a, st);
    }
    return 0;
}

int pick_e(int L) {
    // samples per lane per row; override for tuning with OFS_FAST_E=2|4|8
    static int forced = -1;
    if (forced < 0) {
        const char* s = getenv("OFS_FAST_E");
        forced = s ? atoi(s) : 0;
    }
    if (forced == 2 || forced == 4 || forced == 8) return (L % (64 * forced) == 0) ? forced : 0;
    for (int e : {8, 4, 2})
        if (L % (64 * e) == 0) return e;
    return 0;
}

}  // namespace

int ofs_aa_fast_try(int fmt, int precision, int n_ant, const AaFastArgs& a, hipStream_t st) {
    if (fmt != OFS_C64 || precision != OFS_FP32) return 0;
    if (n_ant < 1 || n_ant > 2) return 0;
    if (a.T < 2 || a.T > TMAX || (a.T & 1)) return 0;
    if (a.L < 128 || a.L > TMAX) return 0;
    const int E = pick_e(a.L);
    if (!E) return 0;
    const int mr = a.L / (64 * E);
    return n_ant == 1 ? launch_e<1>(E, mr, a, st) : launch_e<2>(E, mr, a, st);
}
