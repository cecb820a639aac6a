// postproc.hip — detection post-processing on the GPU: the reference's timing decisions taken
// from metric streams without copying the metrics back to the host.
//
//   trailing_avg_kernel   minn._trailing_average / combined_sc_min._trailing_average
//                         (minn.py:115-128): the reference's float64 recursion, in order
//   plateau_kernel        sc.find_plateau_end_from_metric (sc.py:81-146)
//   minn_peak_kernel      minn.find_minn_peak (minn.py:131-205), on the trailing average
//   sc_gate_kernel        the S&C gate of combined_sc_min.run_simulation (combined_sc_min.py:337-358)
//   segment_peak_kernel   combined_sc_min.find_minn_peak + _streaming_peak_detector
//                         (combined_sc_min.py:183-259), on the trailing average
//
// Layout: metrics [B][n] (f32 or f64 in, f64 smoothed out), one workgroup (or one wave) per
// stream.  Every decision (argmax with first-index ties, first index below a level, runs of a
// mask) is a block reduction or an ordered chunk scan, so the integer answers equal the
// reference's on the same metric values.  Arithmetic that feeds a comparison (0.95·max,
// 0.6·peak, M/max, thr·max, the running sums) is the reference's own float64 expression.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ofdmsync.h"
#include "ofs_common.h"

namespace {

constexpr int PW = 256;                          // threads per workgroup (per stream)
constexpr int64_t NONE = INT64_MAX;

template <class T>
__device__ __forceinline__ double ld(const T* p, int64_t i) { return (double)p[i]; }

// ---- block reductions (256 threads) -------------------------------------------------------
struct Red {
    double v[PW / 64];
    int64_t i[PW / 64];
    int64_t a[PW];
    int64_t b[PW];
};

// argmax with the smallest index on ties (np.argmax); v = -inf / i = NONE for empty lanes
__device__ void block_argmax(double& v, int64_t& i, Red& r) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(v, off, 64);
        const int64_t oi = __shfl_xor(i, off, 64);
        if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
    }
    if (lane == 0) { r.v[w] = v; r.i[w] = i; }
    __syncthreads();
    v = r.v[0]; i = r.i[0];
    for (int k = 1; k < PW / 64; ++k)
        if (r.v[k] > v || (r.v[k] == v && r.i[k] < i)) { v = r.v[k]; i = r.i[k]; }
    __syncthreads();
}

__device__ int64_t block_min(int64_t x, Red& r) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = min(x, (int64_t)__shfl_xor(x, off, 64));
    if (lane == 0) r.i[w] = x;
    __syncthreads();
    int64_t m = r.i[0];
    for (int k = 1; k < PW / 64; ++k) m = min(m, r.i[k]);
    __syncthreads();
    return m;
}

// Runs of a predicate over [lo, hi): thread t owns a contiguous chunk and learns, through a
// suffix-min of per-chunk first-false positions, the next false position after its chunk; it
// then walks its chunk right to left and calls visit(start, end) for every run that STARTS in
// it (end = first false after start, or hi).  Run starts are processed in no particular
// order across threads; callers reduce.
template <class Pred, class Visit>
__device__ void for_each_run(int64_t lo, int64_t hi, Pred pred, Visit visit, Red& r) {
    const int t = threadIdx.x;
    const int64_t len = hi - lo;
    const int64_t C = (len + PW - 1) / PW;
    const int64_t c0 = lo + t * C, c1 = min(hi, c0 + C);
    int64_t ff = hi;                                   // first false in my chunk
    for (int64_t j = c0; j < c1; ++j)
        if (!pred(j)) { ff = j; break; }
    r.a[t] = ff;
    __syncthreads();
    // inclusive suffix min over chunks (Hillis-Steele, 8 steps)
    for (int d = 1; d < PW; d <<= 1) {
        const int64_t o = (t + d < PW) ? r.a[t + d] : hi;
        __syncthreads();
        r.a[t] = min(r.a[t], o);
        __syncthreads();
    }
    int64_t nf = (t + 1 < PW) ? r.a[t + 1] : hi;       // next false after my chunk
    __syncthreads();
    bool cur = false;
    for (int64_t j = c1 - 1; j >= c0; --j) {
        cur = pred(j);
        if (!cur) { nf = j; continue; }
        const bool prev = (j > lo) && pred(j - 1);
        if (!prev) visit(j, nf);
    }
}

// ------------------------------------------------------------------------------------------
// trailing average: one wave per stream; 64 samples are loaded per step and walked in order
// with the running sum on wave-uniform values (only the two-add chain is serial).
// ------------------------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(PW) void trailing_avg_kernel(const T* x, int64_t B, int64_t n, int win,
                                                          int clip, double* y) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * (PW / 64) + (threadIdx.x >> 6);
    if (b >= B) return;
    const T* xs = x + b * n;
    double* ys = y + b * n;
    auto val = [&](int64_t i) {
        const double v = ld(xs, i);
        return (clip && !(v >= 0.0)) ? (v != v ? v : 0.0) : v;    // np.maximum(v, 0.0), NaN kept
    };
    if (win <= 1) {
        for (int64_t i = lane; i < n; i += 64) ys[i] = val(i);
        return;
    }
    double acc = 0.0;
    for (int64_t base = 0; base < n; base += 64) {
        const int64_t i = base + lane;
        const double v = i < n ? val(i) : 0.0;
        const double old = (i < n && i >= win) ? val(i - win) : 0.0;
        const int cnt = (int)min((int64_t)64, n - base);
        double out = 0.0;
        for (int j = 0; j < cnt; ++j) {
            const int64_t idx = base + j;
            acc += ofs::readlane(v, j);                          // minn.py:123
            if (idx >= win) acc -= ofs::readlane(old, j);        // :124-125
            const double den = idx >= win - 1 ? (double)win : (double)(idx + 1);
            const double q = acc / den;                          // :126-127
            if (lane == j) out = q;
        }
        if (i < n) ys[i] = out;
    }
}

// ------------------------------------------------------------------------------------------
// sc.find_plateau_end_from_metric.  Ms = np.convolve(M, ones(w)/w, "same"): length
// Lo = max(n, w), Ms[i] = Σ_j M[j]·(1/w) over j in [i+off-w+1, i+off] ∩ [0, n),
// off = (min(n, w) - 1) // 2 (numpy's "same" centring).
// ------------------------------------------------------------------------------------------
struct PlArgs {
    const void* M; int64_t B, n; int cp, lookahead, w;
    double* Ms; int64_t* out; int32_t* status;
};

// Python slice a[start:stop] on length n (step 1) -> [s, e)
__device__ __forceinline__ void pyslice(int64_t n, int64_t start, int64_t stop, int64_t& s, int64_t& e) {
    if (start < 0) start += n;
    if (stop < 0) stop += n;
    s = start < 0 ? 0 : (start > n ? n : start);
    e = stop < 0 ? 0 : (stop > n ? n : stop);
    if (e < s) e = s;
}

template <class T>
__global__ __launch_bounds__(PW) void plateau_kernel(PlArgs a) {
#pragma clang fp contract(off)
    __shared__ Red r;
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int64_t n = a.n;
    const int w = a.w < 1 ? 1 : a.w;
    const int64_t Lo = n > w ? n : w;
    const T* M = static_cast<const T*>(a.M) + b * n;
    double* Ms = a.Ms + b * Lo;
    if (n == 0) {                                               // sc.py:94-95
        if (t == 0) { a.out[b] = 0; a.status[b] = 0; }
        return;
    }
    const int64_t off = ((n < w ? n : w) - 1) / 2;
    const double vw = 1.0 / (double)w;
    // (a) smoothed metric + first argmax
    double bv = -INFINITY;
    int64_t bi = NONE;
    for (int64_t i = t; i < Lo; i += PW) {
        const int64_t j0 = max((int64_t)0, i + off - w + 1), j1 = min(n - 1, i + off);
        double s = 0.0;
        for (int64_t j = j0; j <= j1; ++j) s += ld(M, j) * vw;
        Ms[i] = s;
        if (s > bv) { bv = s; bi = i; }
    }
    block_argmax(bv, bi, r);                                     // syncs: Ms visible to the block
    const int64_t center = bi;
    const double mcen = Ms[center];
    int64_t res = NONE;
    int32_t br = 0;
    // (b) first index in [center, center + cp) at or below 95 % of the maximum (sc.py:106-114)
    const int64_t post_hi = min(Lo, center + (int64_t)a.cp);
    if (post_hi > center + 1) {
        const double thr_local = 0.95 * mcen;
        int64_t f = NONE;
        for (int64_t j = center + t; j < post_hi; j += PW)
            if (Ms[j] <= thr_local) { f = j; break; }
        f = block_min(f, r);
        if (f != NONE) { res = f; br = 1; }
    }
    // (c) right edge of the earliest run of length >= max(8, cp/2) above 60 % (sc.py:117-133)
    if (res == NONE) {
        const int64_t min_run = max((int64_t)8, (int64_t)(a.cp / 2));
        const double peak = mcen;                                // == max(Ms)
        if (peak > 0) {
            const double thr = 0.6 * peak;
            int64_t best = NONE, best_end = 0;
            for_each_run(0, Lo, [&](int64_t j) { return Ms[j] >= thr; },
                         [&](int64_t s, int64_t e) { if (e - s >= min_run && s < best) { best = s; best_end = e; } }, r);
            const int64_t s_min = block_min(best, r);
            if (s_min != NONE) {
                if (best == s_min) r.b[0] = best_end - 1;
                __syncthreads();
                res = r.b[0]; br = 2;
                __syncthreads();
            }
        }
    }
    // (d) slope fallback around the maximum (sc.py:136-146), with Python slice semantics
    if (res == NONE) {
        const int64_t L = a.lookahead < 0 ? (int64_t)(a.cp / 4) : (int64_t)(a.lookahead > 1 ? a.lookahead : 1);
        const int64_t lo = max((int64_t)0, center - a.cp);
        const int64_t hi = min(Lo - L - 1, center + a.cp);
        int64_t ws, we, as, ae;
        pyslice(Lo, lo, hi, ws, we);
        pyslice(Lo, lo + L, hi + L, as, ae);
        const int64_t nw = we - ws, na = ae - as;
        if (nw != na && nw != 1 && na != 1) {                    // numpy cannot broadcast: ValueError
            if (t == 0) { a.out[b] = -1; a.status[b] = -3; }
            return;
        }
        const int64_t nd = nw == na ? nw : (nw == 1 ? na : nw);
        if (nd == 0) {
            res = center; br = 4;
        } else {
            double dv = -INFINITY;
            int64_t di = NONE;
            for (int64_t k = t; k < nd; k += PW) {
                const double wv = Ms[ws + (nw == 1 ? 0 : k)], av = Ms[as + (na == 1 ? 0 : k)];
                const double d = wv - av;
                if (d > dv) { dv = d; di = k; }
            }
            block_argmax(dv, di, r);
            res = lo + di + L / 2; br = 3;
        }
    }
    if (t == 0) { a.out[b] = res; a.status[b] = br; }
}

// ------------------------------------------------------------------------------------------
// minn.find_minn_peak on the trailing average Ms (f64 [B][n]).  gate = LONGEST run of
// Ms >= thr·max(Ms) (earliest on ties), cut to [blo, bhi); empty -> global argmax.
// status: 0 ok, -1 empty metric, -2 no positive peak (the reference raises ValueError).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(PW) void minn_peak_kernel(const double* Ms_all, int64_t n, double thr,
                                                       int64_t blo, int64_t bhi, int64_t* peak,
                                                       int64_t* glo, int64_t* ghi, int32_t* status) {
    __shared__ Red r;
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const double* Ms = Ms_all + b * n;
    auto put = [&](int64_t p, int64_t l, int64_t h, int32_t s) {
        if (t == 0) { peak[b] = p; if (glo) glo[b] = l; if (ghi) ghi[b] = h; status[b] = s; }
    };
    if (n == 0) { put(-1, 0, 0, -1); return; }
    double mv = -INFINITY;
    int64_t mi = NONE;
    for (int64_t i = t; i < n; i += PW)
        if (Ms[i] > mv) { mv = Ms[i]; mi = i; }
    block_argmax(mv, mi, r);
    if (!(mv > 0.0)) { put(-1, 0, 0, -2); return; }            // minn.py:151-153
    const double level = thr * mv;                              // :154
    int64_t bl = 0, bs = NONE;                                  // longest run, earliest start
    for_each_run(0, n, [&](int64_t j) { return Ms[j] >= level; },
                 [&](int64_t s, int64_t e) { if (e - s > bl || (e - s == bl && s < bs)) { bl = e - s; bs = s; } }, r);
    // reduce (length desc, start asc): encode as one key
    double key = bs == NONE ? -INFINITY : (double)bl;
    int64_t ks = bs;
    block_argmax(key, ks, r);
    int64_t s = NONE, e = NONE;
    if (ks != NONE && key > 0) { s = ks; e = ks + (int64_t)key; }
    if (s != NONE) { s = max(s, blo); e = min(e, bhi); if (s >= e) s = NONE; }   // :186-193
    if (s == NONE) { put(mi, mi, mi + 1, 0); return; }                          // :195-200
    double pv = -INFINITY;
    int64_t pi = NONE;
    for (int64_t i = s + t; i < e; i += PW)
        if (Ms[i] > pv) { pv = Ms[i]; pi = i; }
    block_argmax(pv, pi, r);                                                    // :202-205
    put(pi, s, e, 0);
}

// ------------------------------------------------------------------------------------------
// S&C gate: mask = M/max >= thr (max > 0) else M >= thr; none -> argmax seeded; span =
// [first, last + 1) of the mask.
// ------------------------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(PW) void sc_gate_kernel(const T* M_all, int64_t n, double thr, uint8_t* mask_all,
                                                     int64_t* span) {
    __shared__ Red r;
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const T* M = M_all + b * n;
    uint8_t* mask = mask_all ? mask_all + b * n : nullptr;
    double mv = -INFINITY;
    int64_t mi = NONE;
    for (int64_t i = t; i < n; i += PW) {
        const double v = ld(M, i);
        if (v > mv) { mv = v; mi = i; }
    }
    block_argmax(mv, mi, r);
    int64_t first = NONE, last = -1;
    for (int64_t i = t; i < n; i += PW) {
        const double v = ld(M, i);
        const bool g = mv > 0 ? (v / mv >= thr) : (v >= thr);
        if (mask) mask[i] = g;
        if (g) { first = min(first, i); last = max(last, i); }
    }
    first = block_min(first, r);
    last = -block_min(-last, r);
    if (first == NONE) {                                         // combined_sc_min.py:347-351
        if (t == 0 && mask && n > 0) mask[mi] = 1;
        first = n > 0 ? mi : 0; last = n > 0 ? mi : -1;
    }
    if (t == 0 && span) { span[2 * b] = first; span[2 * b + 1] = last + 1; }
}

// ------------------------------------------------------------------------------------------
// first-run peak: first argmax (strict >) of Ms over the FIRST run of mask ∩ [blo, bhi).
// status -1: empty gate region (the reference raises ValueError).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(PW) void segment_peak_kernel(const double* Ms_all, const uint8_t* mask_all, int64_t n,
                                                          int64_t blo, int64_t bhi, int64_t* peak, int32_t* status) {
    __shared__ Red r;
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const double* Ms = Ms_all + b * n;
    const uint8_t* mask = mask_all + b * n;
    if (n == 0) { if (t == 0) { peak[b] = 0; status[b] = 0; } return; }    // combined_sc_min.py:223-224
    int64_t s = NONE;
    for (int64_t i = blo + t; i < bhi; i += PW)
        if (mask[i]) { s = i; break; }
    s = block_min(s, r);
    if (s == NONE) { if (t == 0) { peak[b] = -1; status[b] = -1; } return; }
    int64_t e = NONE;
    for (int64_t i = s + t; i < bhi; i += PW)
        if (!mask[i]) { e = i; break; }
    e = min(block_min(e, r), bhi);
    double pv = -INFINITY;
    int64_t pi = NONE;
    for (int64_t i = s + t; i < e; i += PW)
        if (Ms[i] > pv) { pv = Ms[i]; pi = i; }
    block_argmax(pv, pi, r);
    if (t == 0) { peak[b] = pi; status[b] = 0; }
}

bool real_ok(int p) { return p == OFS_FP32 || p == OFS_FP64; }
inline hipError_t last() { return hipGetLastError(); }

}  // namespace

extern "C" {

int32_t ofs_trailing_average(int32_t precision, const void* x, int64_t B, int64_t n, int32_t win,
                             int32_t clip_negative, double* out, void* stream) {
    if (!real_ok(precision) || OFS_MISSING(x, B * n) || OFS_MISSING(out, B * n) || B < 0 || n < 0) return OFS_EINVAL;
    if (B == 0 || n == 0) return OFS_OK;
    const dim3 grid((unsigned)((B + PW / 64 - 1) / (PW / 64)));
    hipStream_t st = (hipStream_t)stream;
    if (precision == OFS_FP64)
        hipLaunchKernelGGL(trailing_avg_kernel<double>, grid, dim3(PW), 0, st, (const double*)x, B, n, win, clip_negative, out);
    else
        hipLaunchKernelGGL(trailing_avg_kernel<float>, grid, dim3(PW), 0, st, (const float*)x, B, n, win, clip_negative, out);
    return last() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_plateau_end(int32_t precision, const void* M, int64_t B, int64_t n, int32_t cp_len,
                        int32_t lookahead, int32_t smooth_win, double* Ms, int64_t* plateau_end,
                        int32_t* status, void* stream) {
    if (!real_ok(precision) || OFS_MISSING(M, B * n) || OFS_MISSING(Ms, B * n) || OFS_MISSING(plateau_end, B) ||
        OFS_MISSING(status, B) || B < 0 || n < 0 || cp_len < 0)
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    if (B > 0x7fffffff) return OFS_EINVAL;
    PlArgs a{M, B, n, cp_len, lookahead, smooth_win, Ms, plateau_end, status};
    hipStream_t st = (hipStream_t)stream;
    if (precision == OFS_FP64) hipLaunchKernelGGL(plateau_kernel<double>, dim3((unsigned)B), dim3(PW), 0, st, a);
    else hipLaunchKernelGGL(plateau_kernel<float>, dim3((unsigned)B), dim3(PW), 0, st, a);
    return last() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_minn_peak(const double* Ms, int64_t B, int64_t n, double gate_threshold, int64_t bound_lo,
                      int64_t bound_hi, int64_t* peak, int64_t* gate_lo, int64_t* gate_hi, int32_t* status,
                      void* stream) {
    if (OFS_MISSING(Ms, B * n) || OFS_MISSING(peak, B) || OFS_MISSING(status, B) || B < 0 || n < 0 || B > 0x7fffffff)
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipLaunchKernelGGL(minn_peak_kernel, dim3((unsigned)B), dim3(PW), 0, (hipStream_t)stream, Ms, n,
                       gate_threshold, bound_lo, bound_hi, peak, gate_lo, gate_hi, status);
    return last() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_sc_gate(int32_t precision, const void* M_sc, int64_t B, int64_t n, double threshold,
                    uint8_t* mask, int64_t* span, void* stream) {
    if (!real_ok(precision) || OFS_MISSING(M_sc, B * n) || B < 0 || n < 0 || B > 0x7fffffff || (!mask && !span && B > 0))
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipStream_t st = (hipStream_t)stream;
    if (precision == OFS_FP64)
        hipLaunchKernelGGL(sc_gate_kernel<double>, dim3((unsigned)B), dim3(PW), 0, st, (const double*)M_sc, n, threshold, mask, span);
    else
        hipLaunchKernelGGL(sc_gate_kernel<float>, dim3((unsigned)B), dim3(PW), 0, st, (const float*)M_sc, n, threshold, mask, span);
    return last() == hipSuccess ? OFS_OK : OFS_EHIP;
}

int32_t ofs_segment_peak(const double* Ms, const uint8_t* mask, int64_t B, int64_t n, int64_t bound_lo,
                         int64_t bound_hi, int64_t* peak, int32_t* status, void* stream) {
    if ((!Ms || !mask) && n > 0 && B > 0) return OFS_EINVAL;
    if (OFS_MISSING(peak, B) || OFS_MISSING(status, B) || B < 0 || n < 0 || B > 0x7fffffff || bound_lo < 0 || bound_hi > n) return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipLaunchKernelGGL(segment_peak_kernel, dim3((unsigned)B), dim3(PW), 0, (hipStream_t)stream, Ms, mask, n,
                       bound_lo, bound_hi, peak, status);
    return last() == hipSuccess ? OFS_OK : OFS_EHIP;
}

}  // extern "C"
