// ofs_common.h — device helpers shared by the HIP translation units of libofdmsync.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// a required pointer may be null only when the buffer it describes is empty (B = 0, T = 0)
#define OFS_MISSING(p, n) ((p) == nullptr && (int64_t)(n) > 0)

namespace ofs {

// Debug / A-B variants (include/ofdmsync.h ofs_debug_set_variant): unset unless a caller set one
// through that entry point; the table lives in ofdmsync.hip.
enum Variant : int {
    V_EXACT, V_FAST_E, V_FAST_E_DO, V_FAST_SCAN, V_FAST_SCAN_DO, V_RTL_WPB, V_PARK_DIRECT, V_ZW64,
    V_ZW64_GRID, V_ZS, V_ZF_ITEMS, V_ZS_PAIR, V_ZS_DEFER, V_ZS_BPL, V_ZS_C, V_ZS_GBLK, V_MC_FUSED,
    V_MC_FUSE_X, V_ZC_SEQ, V_ZC_NODMA, V_BE_FAST, V_MC_PERS, V_FAST_LDS, V_OCC_LDS, V_COUNT
};
int64_t variant(Variant v);                                     // INT64_MIN when unset
inline bool variant_is(Variant v, int64_t value) { return variant(v) == value; }
inline bool variant_off(Variant v) { return variant(v) == 0; }                 // set to 0
inline bool variant_on(Variant v) { const int64_t x = variant(v); return x != INT64_MIN && x != 0; }
inline int64_t variant_or(Variant v, int64_t dflt) { const int64_t x = variant(v); return x == INT64_MIN ? dflt : x; }
// variant OCC_LDS: bytes of unused dynamic LDS added to a wave-per-stream launch (occupancy-cap A/B
// of the memory-bound kernels; 0 / unset = none)
inline size_t occ_lds() { const int64_t x = variant(V_OCC_LDS); return x > 0 && x <= 65536 ? (size_t)x : 0; }


// ---- cross-lane (wave64) helpers: DPP row shifts + row broadcasts (GFX9-family DPP) ----
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = dpp_i<CTRL>(__double2loint(v));
    const int hi = dpp_i<CTRL>(__double2hiint(v));
    return __hiloint2double(hi, lo);
}

// inclusive wave64 prefix sum of doubles (rocPRIM-style gfx9 DPP ladder)
__device__ __forceinline__ double wave_scan_add(double v, int lane) {
    const int rl = lane & 15;
    double t;
    t = dpp_d<0x111>(v); if (rl >= 1) v += t;          // row_shr:1
    t = dpp_d<0x112>(v); if (rl >= 2) v += t;          // row_shr:2
    t = dpp_d<0x114>(v); if (rl >= 4) v += t;          // row_shr:4
    t = dpp_d<0x118>(v); if (rl >= 8) v += t;          // row_shr:8
    t = dpp_d<0x142>(v); if ((lane & 31) >= 16) v += t; // row_bcast:15
    t = dpp_d<0x143>(v); if (lane >= 32) v += t;        // row_bcast:31
    return v;
}

// inclusive wave64 prefix max of ints
__device__ __forceinline__ int wave_scan_max(int v, int lane) {
    const int rl = lane & 15;
    int t;
    t = dpp_i<0x111>(v); if (rl >= 1) v = max(v, t);
    t = dpp_i<0x112>(v); if (rl >= 2) v = max(v, t);
    t = dpp_i<0x114>(v); if (rl >= 4) v = max(v, t);
    t = dpp_i<0x118>(v); if (rl >= 8) v = max(v, t);
    t = dpp_i<0x142>(v); if ((lane & 31) >= 16) v = max(v, t);
    t = dpp_i<0x143>(v); if (lane >= 32) v = max(v, t);
    return v;
}

// value of lane-1 (wave_shr:1); lane 0 gets `first`
__device__ __forceinline__ double wave_shr1(double v, int lane, double first) {
    const double t = dpp_d<0x138>(v);
    return lane == 0 ? first : t;
}
__device__ __forceinline__ int wave_shr1(int v, int lane, int first) {
    const int t = dpp_i<0x138>(v);
    return lane == 0 ? first : t;
}

__device__ __forceinline__ double readlane(double v, int j) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float readlane(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}
__device__ __forceinline__ int readlane(int v, int j) { return __builtin_amdgcn_readlane(v, j); }

// full wave64 reductions by a DPP ladder (row_shr 1/2/4/8, row_bcast 15/31): lanes without a
// source keep the identity (bound_ctrl off, old = identity); the result is read from lane 63
template <int CTRL, int RMASK = 0xf>
__device__ __forceinline__ int dpp_old(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, RMASK, 0xf, false);
}
template <class Op>
__device__ __forceinline__ int dpp_reduce_bits(int v, int ident, Op op) {
    v = op(v, dpp_old<0x111>(ident, v));
    v = op(v, dpp_old<0x112>(ident, v));
    v = op(v, dpp_old<0x114>(ident, v));
    v = op(v, dpp_old<0x118>(ident, v));
    v = op(v, dpp_old<0x142, 0xa>(ident, v));
    v = op(v, dpp_old<0x143, 0xc>(ident, v));
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ float wave_max(float v) {
    const int r = dpp_reduce_bits(__float_as_int(v), __float_as_int(-__builtin_huge_valf()), [](int a, int b) {
        return __float_as_int(fmaxf(__int_as_float(a), __int_as_float(b)));
    });
    return __int_as_float(r);
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
    return dpp_reduce_bits(v, INT32_MIN, [](int a, int b) { return max(a, b); });
}
__device__ __forceinline__ int wave_min(int v) {
    return dpp_reduce_bits(v, INT32_MAX, [](int a, int b) { return min(a, b); });
}

// XCD-aware block order.  The dispatcher deals workgroups round-robin over the 8 XCDs (each
// with its own L2 and TLB), so consecutive blockIdx land on different XCDs.  Remapped, XCD x
// walks the contiguous block range [x·n/8, (x+1)·n/8) in order: each XCD streams through
// one compact region of every buffer instead of touching pages all over them.  Identity when
// the grid is not a multiple of 8 (OFS_XCD_REMAP=0 at build time disables it for A/B).  Paired
// A/B with one-wave workgroups on the bench's contiguous arena: 1.1-1.7 % faster in 6 of 6
// allocations (with four-wave workgroups it had measured slower).
#ifndef OFS_XCD_REMAP
#define OFS_XCD_REMAP 1
#endif
__device__ __forceinline__ unsigned xcd_block() {
#if OFS_XCD_REMAP
    const unsigned n = gridDim.x, b = blockIdx.x;
    if ((n & 7u) == 0u) return (b & 7u) * (n >> 3) + (b >> 3);
    return b;
#else
    return blockIdx.x;
#endif
}

// the same order for the other wave-per-stream kernels (tuning builds: -DOFS_XCD_WIDE=1)
#ifndef OFS_XCD_WIDE
#define OFS_XCD_WIDE 0
#endif
__device__ __forceinline__ unsigned xcd_block_w() {
#if OFS_XCD_WIDE
    return xcd_block();
#else
    return blockIdx.x;
#endif
}

// atan2 in fp32 to ~1.5e-7 rad: odd degree-15 polynomial on [0, 1] (fitted to atan, fp32
// coefficients) plus octant reduction; ~25 VALU instead of ocml's ~125.  Used where the inputs
// are fp32 results anyway (the fast path's CFO from an fp32 P).
__device__ __forceinline__ float fast_atan2f(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mx > 0.f ? mn * __builtin_amdgcn_rcpf(mx) : 0.f;
    const float s = a * a;
    float r = -0.004054530523717403f;
    r = fmaf(r, s, 0.02186284027993679f);
    r = fmaf(r, s, -0.055912185460329056f);
    r = fmaf(r, s, 0.09642189741134644f);
    r = fmaf(r, s, -0.1390862762928009f);
    r = fmaf(r, s, 0.19946566224098206f);
    r = fmaf(r, s, -0.33329859375953674f);
    r = fmaf(r, s, 0.9999993443489075f);
    r *= a;
    if (ay > ax) r = 1.5707963267948966f - r;
    if (x < 0.f) r = 3.141592653589793f - r;
    return __builtin_copysignf(r, y);
}

// zero-filled DPP move (bound_ctrl): lanes without a source read 0
template <int CTRL, int RMASK = 0xf>
__device__ __forceinline__ double dppz(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, RMASK, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, RMASK, 0xf, true);
    return __hiloint2double(hi, lo);
}
// inclusive wave64 prefix sum with zero-filled moves (no lane predicates)
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

// the same ladder on 32-bit integers (one v_add with a DPP source per step; exact)
template <int CTRL, int RMASK = 0xf>
__device__ __forceinline__ int dppz_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, RMASK, 0xf, true);
}
__device__ __forceinline__ int scan_add_i32(int v) {
    v += dppz_i<0x111>(v);
    v += dppz_i<0x112>(v);
    v += dppz_i<0x114>(v);
    v += dppz_i<0x118>(v);
    v += dppz_i<0x142, 0xa>(v);
    v += dppz_i<0x143, 0xc>(v);
    return v;
}

// the same ladder on floats (one v_add_f32 with a DPP source per step)
template <int CTRL, int RMASK = 0xf>
__device__ __forceinline__ float dppz_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, RMASK, 0xf, true));
}
__device__ __forceinline__ float scan_add_f32(float v) {
    v += dppz_f<0x111>(v);
    v += dppz_f<0x112>(v);
    v += dppz_f<0x114>(v);
    v += dppz_f<0x118>(v);
    v += dppz_f<0x142, 0xa>(v);
    v += dppz_f<0x143, 0xc>(v);
    return v;
}

// Scan of one lane value across a row (the wave): x = sum over lanes < l, u = sum over lanes > l,
// tot = the row total.  F32 = false: fp64 ladder (x, u exact to fp32 rounding, tot exact);
// F32 = true: fp32 ladder, 6 rounded adds deep: the sums are of one row's lane totals only (no
// cancellation against a stream-wide prefix), so |dx|, |dtot| <= 6u·Σ_row|v| and |du| <= 13u·Σ_row|v|
// (the detect-only kernel: half the issue slots of the fp64 ladder, r03f).
struct RowScan { float x, u; double tot; };
template <bool F32>
__device__ __forceinline__ RowScan row_scan(float v) {
    if constexpr (F32) {
        const float i = scan_add_f32(v);
        const float t = readlane(i, 63);
        return RowScan{dppz_f<0x138>(i), t - i, (double)t};
    } else {
        const double i = scan_add((double)v);
        const double t = readlane(i, 63);
        return RowScan{(float)shr1z(i), (float)(t - i), t};
    }
}


// One LDS-DMA: lane l's 16 bytes at g -> LDS[lds + 16 l] (64 lanes = 1 KiB), issued as inline asm.
// Through __builtin_amdgcn_global_load_lds the compiler cannot tell which LDS the DMA writes, so
// it guards every later LDS read with vmcnt(0) (and implements a "local" release fence as
// vmcnt(0)), draining DMAs meant to stay in flight - and, in waves that also store to global
// memory, those stores.  Callers order the DMAs themselves: s_waitcnt vmcnt(n) in the issuing wave
// before the data is read (and a barrier before other waves read it).
__device__ __forceinline__ void lds_dma16(const void* g, const void* lds) {
    const uint32_t m = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m) : "memory", "m0");
}


// s_waitcnt vmcnt(n) for an n that folds to a constant at compile time (unrolled loops); n > 63
// waits for the hardware maximum (63), i.e. at least as long
#define OFS_VMW(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
__device__ __forceinline__ void vmcnt_wait(int n) {
    switch (n < 63 ? n : 63) {
        OFS_VMW(0) OFS_VMW(1) OFS_VMW(2) OFS_VMW(3) OFS_VMW(4) OFS_VMW(5) OFS_VMW(6) OFS_VMW(7)
        OFS_VMW(8) OFS_VMW(9) OFS_VMW(10) OFS_VMW(11) OFS_VMW(12) OFS_VMW(13) OFS_VMW(14) OFS_VMW(15)
        OFS_VMW(16) OFS_VMW(17) OFS_VMW(18) OFS_VMW(19) OFS_VMW(20) OFS_VMW(21) OFS_VMW(22) OFS_VMW(23)
        OFS_VMW(24) OFS_VMW(25) OFS_VMW(26) OFS_VMW(27) OFS_VMW(28) OFS_VMW(29) OFS_VMW(30) OFS_VMW(31)
        OFS_VMW(32) OFS_VMW(33) OFS_VMW(34) OFS_VMW(35) OFS_VMW(36) OFS_VMW(37) OFS_VMW(38) OFS_VMW(39)
        OFS_VMW(40) OFS_VMW(41) OFS_VMW(42) OFS_VMW(43) OFS_VMW(44) OFS_VMW(45) OFS_VMW(46) OFS_VMW(47)
        OFS_VMW(48) OFS_VMW(49) OFS_VMW(50) OFS_VMW(51) OFS_VMW(52) OFS_VMW(53) OFS_VMW(54) OFS_VMW(55)
        OFS_VMW(56) OFS_VMW(57) OFS_VMW(58) OFS_VMW(59) OFS_VMW(60) OFS_VMW(61) OFS_VMW(62)
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
}
#undef OFS_VMW

}  // namespace ofs

// internal launchers implemented in aa_fast.hip (C++ linkage, not part of the ABI)
struct AaFastArgs {
    const void* x;
    int64_t B, T;
    int32_t L;
    void* P; void* R; void* M; uint8_t* valid;
    int32_t detect; double thr; int32_t hyst; double fs;
    int32_t max_ev; int32_t* n_ev; int64_t* ev_i; double* ev_r;
};
// returns 1 if the fast path handled the call (launched), 0 if not applicable, <0 on error
int ofs_aa_fast_try(int fmt, int precision, int n_ant, const AaFastArgs& a, hipStream_t st);
// 10*E + MR of the fast kernel a shape dispatches to, 0 if the general engine handles it
int ofs_aa_fast_plan(int fmt, int precision, int n_ant, int64_t T, int L);

// integer-exact wave-per-stream paths for int16 I/Q input (aa_exact.hip): 10*E + MR (or MW) of
// the kernel a shape dispatches to, 0 if the general engine handles it; *_try returns 1 if
// launched, 0 if not covered, <0 on error
int ofs_aa_exact_plan(int fmt, int precision, int n_ant, int64_t T, int L);
int ofs_aa_exact_try(int fmt, int precision, int n_ant, const AaFastArgs& a, hipStream_t st);
struct RtlExactCall {
    const void* x; int64_t B, T; int32_t Q;
    int32_t shift, smooth_mode, frac_bits; double thr_value;
    double* corr_total; double* corr_positive; double* smooth; double* energy_total;
    double* corr_scaled; double* energy_scaled; uint8_t* mvalid; uint8_t* above;
    int32_t detect, hyst, toff, max_ev; int32_t* n_ev; int64_t* ev; int64_t* open_start;
};
int ofs_rtl_exact_plan(int fmt, int n_br, int64_t T, int Q);
int ofs_rtl_exact_try(int fmt, int n_br, const RtlExactCall& c, hipStream_t st);

// streaming fast path of the S&C / combined S&C / Minn window metrics (win_fast.hip)
struct WinFastArgs {
    const void* x; int64_t B, T; int N;
    void* M; void* P; void* R;
};
// mode: 1 S&C (sc.py), 2 combined S&C (combined_sc_min.py), 3 Minn.  Returns 1 if launched,
// 0 if the shape is not covered (caller uses the general engine), <0 on error.
int ofs_win_fast_try(int mode, int fmt, int precision, int n_br, const WinFastArgs& a, hipStream_t st);
int ofs_win_fast_plan(int mode, int fmt, int precision, int n_br, int64_t T, int N);
// fused combined S&C + Minn (one pass): 10*E + MW, or 0
int ofs_sc_minn_fast_plan(int fmt, int precision, int n_br, int64_t T, int N);
int ofs_sc_minn_fast_try(int fmt, int precision, int n_br, const void* x, int64_t B, int64_t T, int N,
                         void* Ms, void* Ps, void* Rs, void* Mm, void* Pm, void* Rm, hipStream_t st);
