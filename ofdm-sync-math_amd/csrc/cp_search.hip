// cp_search.hip — CP-correlation searches around an estimated CP start (core.py:199-336):
//
//   mode 0 (OFS_CPS_ROBUST): Σ_d P_win(d) over d in [est - span, est + span) ∩ valid, angle -> CFO
//                            (core.estimate_cfo_from_cp_robust, core.py:199-231)
//   mode 1 (OFS_CPS_PEAK):   d* = first argmax_d |P_cp(d)| (strict >), CFO from P_cp(d*)
//                            (estimate_cfo_from_cp_peak / _with_index, core.py:234-303;
//                            find_cp_start_via_corr, core.py:306-336, is d* with span = search_half)
//
// with P_w(d) = Σ_br Σ_{n<w} x[d+n]·conj(x[d+n+N]).  One workgroup per stream; every thread owns
// a strided set of offsets d and sums its windows directly in fp64 (no prefix differences, so
// |P(d)| has no cancellation error beyond the reference's own), then a block reduction.
// The search range is the reference's: d_lo = max(0, est - span),
// d_hi = min(T - (N + w), est + span); an empty range is reported as status 1 (the reference
// falls back to estimate_cfo_from_cp at est; the caller does the same with ofs_cp_cfo).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "ofdmsync.h"
#include "ofs_common.h"

namespace {

constexpr int SW = 256;

template <int FMT>
__device__ __forceinline__ double2 ldc(const void* p, int64_t i) {
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

struct CpsArgs {
    const void* x; int64_t T; int nb; const int64_t* est;
    int N, w, span, mode; double fs;
    double* P; int64_t* d; double* cfo; int32_t* status;
};

template <int FMT>
__global__ __launch_bounds__(SW) void cp_search_kernel(CpsArgs a) {
    __shared__ double sv[SW / 64][3];
    __shared__ int64_t si[SW / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t b = blockIdx.x;
    const int64_t est = a.est[b];
    const int64_t d_lo = max((int64_t)0, est - a.span);
    const int64_t d_hi = min(a.T - ((int64_t)a.N + a.w), est + a.span);
    if (d_hi <= d_lo) {                                   // core.py:222-223, :254-255
        if (t == 0) {
            a.status[b] = 1;
            if (a.d) a.d[b] = est;
            a.cfo[b] = NAN;
            if (a.P) { a.P[2 * b] = NAN; a.P[2 * b + 1] = NAN; }
        }
        return;
    }
    auto window = [&](int64_t d, double& pr, double& pi) {
        pr = 0.0; pi = 0.0;
        for (int br = 0; br < a.nb; ++br) {
            const int64_t row = (b * a.nb + br) * a.T;
            for (int n = 0; n < a.w; ++n) {
                const double2 u = ldc<FMT>(a.x, row + d + n);
                const double2 v = ldc<FMT>(a.x, row + d + n + a.N);
                pr += u.x * v.x + u.y * v.y;              // u * conj(v)
                pi += u.y * v.x - u.x * v.y;
            }
        }
    };
    double br_ = 0.0, bi_ = 0.0, key = -1.0;
    int64_t bd = INT64_MAX;
    for (int64_t d = d_lo + t; d < d_hi; d += SW) {
        double pr, pi;
        window(d, pr, pi);
        if (a.mode == 0) {
            br_ += pr; bi_ += pi;                         // core.py:225-228
        } else {
            const double mag = hypot(pr, pi);              // float(np.abs(P)), core.py:261-265
            if (mag > key) { key = mag; bd = d; br_ = pr; bi_ = pi; }
        }
    }
    if (a.mode == 0) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            br_ += __shfl_xor(br_, off, 64);
            bi_ += __shfl_xor(bi_, off, 64);
        }
        if (lane == 0) { sv[wv][0] = br_; sv[wv][1] = bi_; }
        __syncthreads();
        if (t == 0) {
            double r = 0.0, i = 0.0;
            for (int k = 0; k < SW / 64; ++k) { r += sv[k][0]; i += sv[k][1]; }
            br_ = r; bi_ = i; bd = est;
        }
    } else {                                              // first argmax: larger |P|, then smaller d
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double ok = __shfl_xor(key, off, 64);
            const int64_t od = __shfl_xor(bd, off, 64);
            const double orr = __shfl_xor(br_, off, 64), oi = __shfl_xor(bi_, off, 64);
            if (ok > key || (ok == key && od < bd)) { key = ok; bd = od; br_ = orr; bi_ = oi; }
        }
        if (lane == 0) { sv[wv][0] = key; sv[wv][1] = br_; sv[wv][2] = bi_; si[wv] = bd; }
        __syncthreads();
        if (t == 0) {
            for (int k = 1; k < SW / 64; ++k)
                if (sv[k][0] > sv[0][0] || (sv[k][0] == sv[0][0] && si[k] < si[0])) {
                    sv[0][0] = sv[k][0]; sv[0][1] = sv[k][1]; sv[0][2] = sv[k][2]; si[0] = si[k];
                }
            br_ = sv[0][1]; bi_ = sv[0][2]; bd = si[0];
        }
    }
    if (t == 0) {
        a.status[b] = 0;
        if (a.d) a.d[b] = bd;
        if (a.P) { a.P[2 * b] = br_; a.P[2 * b + 1] = bi_; }
        a.cfo[b] = -atan2(bi_, br_) * a.fs / (2.0 * M_PI * (double)a.N);   // core.py:229-230
    }
}

}  // namespace

extern "C" int32_t ofs_cp_search(int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                                 const int64_t* est, int32_t n_fft, int32_t win_len, int32_t span,
                                 int32_t mode, double fs_hz, double* P_out, int64_t* d_out,
                                 double* cfo_out, int32_t* status, void* stream) {
    if (!(in_fmt == OFS_C64 || in_fmt == OFS_C128 || in_fmt == OFS_CI16) || OFS_MISSING(x, B * T) || OFS_MISSING(est, B) ||
        OFS_MISSING(cfo_out, B) || OFS_MISSING(status, B) || B < 0 || n_br < 1 || T < 0 || n_fft < 0 || win_len < 1 || span < 0 ||
        (mode != 0 && mode != 1) || B > 0x7fffffff)
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    CpsArgs a{x, T, n_br, est, n_fft, win_len, span, mode, fs_hz, P_out, d_out, cfo_out, status};
    hipStream_t st = (hipStream_t)stream;
    switch (in_fmt) {
        case OFS_C64: hipLaunchKernelGGL(cp_search_kernel<OFS_C64>, dim3((unsigned)B), dim3(SW), 0, st, a); break;
        case OFS_C128: hipLaunchKernelGGL(cp_search_kernel<OFS_C128>, dim3((unsigned)B), dim3(SW), 0, st, a); break;
        default: hipLaunchKernelGGL(cp_search_kernel<OFS_CI16>, dim3((unsigned)B), dim3(SW), 0, st, a); break;
    }
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}
