// zc_rocfft.hip — the rocFFT leg of zc_freq.compute_frequency_metric (zc_freq.py:62-99).
//
// The north-star formulation of the ZC frequency-domain path: one library FFT per window
// (rocFFT, batched over every stream x branch of one offset) followed by a hand-written
// gather / conj-multiply / |.|^2 / normalise kernel, and a first-argmax kernel for the
// reference's `peak_index = int(np.argmax(metric))` (zc_freq.py:144).
//
// It is the comparison path for the fused window-FFT kernel of corr.hip (zc_win64_kernel):
// rocFFT must write the whole N-point spectrum of every window (8 B/bin fp32) and the gather
// reads 62 bins of it back, so per window it moves 2 x 8N bytes against the fused kernel's
// 8N (SURVEY §8d "report both").  Both are measured by tools/bench_configs.py (cfg5 / cfg5_rocfft).
//
// Index convention: the reference takes bins = fftshift(X)[(N/2 + idx) % N]; fftshift is
// roll(X, N//2), so bin k is X[((N/2 + idx_k) % N - N//2) mod N] of the unshifted spectrum.
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>
#include <stdint.h>
#include <math.h>
#include <mutex>
#include <string.h>
#include "ofdmsync.h"

namespace {

constexpr int ZB = 64;          // max template bins (one lane each)
constexpr int ZWG = 256;        // 4 waves = 4 streams per workgroup

// Pruned output (store callback): rocFFT hands every output element to zc_store_cb instead of
// writing it; the callback keeps only the template bins, in a compact [n_windows][n_bins]
// buffer, so the dense N-point spectrum never reaches HBM (2 x 8N -> 8N + 8 n_bins bytes per
// window).  cbdata lives in device memory; slot[k] = template position of unshifted bin k or -1.
struct ZcCbData {
    void* compact;              // [n_windows][n_bins] c64 | c128
    int32_t n_bins, log2N;
    int64_t row_T, n_off;       // rows plans: windows w with w % row_T >= n_off straddle two rows (dropped)
    int16_t slot[4096];
};

__device__ __forceinline__ bool zc_cb_keep(const ZcCbData* d, size_t w) {
    return d->row_T == 0 || (int64_t)(w % (size_t)d->row_T) < d->n_off;
}
__device__ void zc_store_cb_f32(void* data, size_t offset, float2 element, void* cbdata, void*) {
    (void)data;
    const ZcCbData* d = static_cast<const ZcCbData*>(cbdata);
    const size_t k = offset & ((size_t(1) << d->log2N) - 1);
    const int s = d->slot[k];
    const size_t w = offset >> d->log2N;
    if (s >= 0 && zc_cb_keep(d, w)) static_cast<float2*>(d->compact)[w * d->n_bins + s] = element;
}
__device__ void zc_store_cb_f64(void* data, size_t offset, double2 element, void* cbdata, void*) {
    (void)data;
    const ZcCbData* d = static_cast<const ZcCbData*>(cbdata);
    const size_t k = offset & ((size_t(1) << d->log2N) - 1);
    const int s = d->slot[k];
    const size_t w = offset >> d->log2N;
    if (s >= 0 && zc_cb_keep(d, w)) static_cast<double2*>(d->compact)[w * d->n_bins + s] = element;
}
__device__ void* zc_store_cb_f32_ptr = (void*)zc_store_cb_f32;
__device__ void* zc_store_cb_f64_ptr = (void*)zc_store_cb_f64;

struct ZcFftPlan {
    rocfft_plan plan = nullptr;     // `chunk` windows per execution
    rocfft_plan tail = nullptr;     // the last n_windows % chunk windows (chunked plans only)
    int64_t chunk = 0;              // windows per rocFFT execution (= n_windows unless chunked)
    int32_t precision = 0;
    int32_t N = 0;
    int64_t n_windows = 0;
    int64_t in_dist = 0;
    size_t work_bytes = 0;
    int32_t prune = 0;          // > 0: pruned output with this many bins (store callback)
    ZcCbData* cb_dev = nullptr; // device copy of the callback data
    ZcCbData* cb_host = nullptr;// pinned staging
    void* cb_fn = nullptr;      // device address of the store callback
    // rows plan (ofs_zc_fft_plan_create_rows): every offset of `rows` consecutive [T]-sample rows in ONE
    // execution - windows at distance 1 sample from sample cp of the first row
    int64_t rows = 0;           // rows per execution (0: the per-offset plan above)
    int64_t row_T = 0, n_off = 0;
    int32_t cp = 0;
};

struct GatherArgs {
    const void* spec;           // [B][n_br][N] c64 | c128 (unshifted spectrum of one offset)
    int64_t B, n_off, off, b0;  // B streams of this execution, the first being stream b0
    int32_t n_br, N, n_bins;
    double e_t;
    void* metric;               // [B][n_off] f32 | f64
    int32_t pos[ZB];            // unshifted spectrum index of template bin k
    double t_re[ZB], t_im[ZB];  // template bins
};

// One wave per stream: lane k owns template bin k; sum_br vdot(t, bins) and sum_br sum |bins|^2
// are accumulated in fp64 (zc_freq.py:88-95) and reduced across the wave.
template <class R>
__global__ __launch_bounds__(ZWG) void zc_gather_kernel(GatherArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * (ZWG / 64) + (threadIdx.x >> 6);
    if (b >= a.B) return;
    double cr = 0.0, ci = 0.0, en = 0.0;
    if (lane < a.n_bins) {
        const int p = a.pos[lane];
        const double tr = a.t_re[lane], ti = a.t_im[lane];
        for (int br = 0; br < a.n_br; ++br) {
            const int64_t i = ((b * a.n_br + br) * (int64_t)a.N + p);
            double xr, xi;
            if constexpr (sizeof(R) == 4) {
                const float2 v = reinterpret_cast<const float2*>(a.spec)[i];
                xr = v.x; xi = v.y;
            } else {
                const double2 v = reinterpret_cast<const double2*>(a.spec)[i];
                xr = v.x; xi = v.y;
            }
            cr += tr * xr + ti * xi;                     // conj(t) * x
            ci += tr * xi - ti * xr;
            en += xr * xr + xi * xi;
        }
    }
    for (int m = 32; m >= 1; m >>= 1) {
        cr += __shfl_xor(cr, m);
        ci += __shfl_xor(ci, m);
        en += __shfl_xor(en, m);
    }
    if (lane == 0) {
        const double v = (cr * cr + ci * ci) / fmax(a.e_t * en, 1e-12);
        if constexpr (sizeof(R) == 4) reinterpret_cast<float*>(a.metric)[(a.b0 + b) * a.n_off + a.off] = (float)v;
        else reinterpret_cast<double*>(a.metric)[(a.b0 + b) * a.n_off + a.off] = v;
    }
}

// rows plans: metric[b][off] for every offset of the execution's streams from the spectrum of windows
// w = (b·n_br + br)·T + off: compact [window][n_bins] (pruned plans) or dense [window][N] (no callback).  One wave per (stream, offset), lane k = template bin k; the
// streams stride over gridDim.y (<= 65535, the launch limit), so any rows-per-execution fits.
template <class R>
__global__ __launch_bounds__(ZWG) void zc_gather_rows_kernel(GatherArgs a, int64_t T) {
    const int lane = threadIdx.x & 63;
    const int64_t off = (int64_t)blockIdx.x * (ZWG / 64) + (threadIdx.x >> 6);
    if (off >= a.n_off) return;
    for (int64_t b = blockIdx.y; b < a.B; b += gridDim.y) {
        double cr = 0.0, ci = 0.0, en = 0.0;
        if (lane < a.n_bins) {
            const double tr = a.t_re[lane], ti = a.t_im[lane];
            for (int br = 0; br < a.n_br; ++br) {
                const int64_t i = ((b * a.n_br + br) * T + off) * a.N + a.pos[lane];   // pruned: N = n_bins, pos = k
                double xr, xi;
                if constexpr (sizeof(R) == 4) {
                    const float2 v = reinterpret_cast<const float2*>(a.spec)[i];
                    xr = v.x; xi = v.y;
                } else {
                    const double2 v = reinterpret_cast<const double2*>(a.spec)[i];
                    xr = v.x; xi = v.y;
                }
                cr += tr * xr + ti * xi;                     // conj(t) * x   (zc_freq.py:88-95)
                ci += tr * xi - ti * xr;
                en += xr * xr + xi * xi;
            }
        }
        for (int m = 32; m >= 1; m >>= 1) {
            cr += __shfl_xor(cr, m);
            ci += __shfl_xor(ci, m);
            en += __shfl_xor(en, m);
        }
        if (lane == 0) {
            const double v = (cr * cr + ci * ci) / fmax(a.e_t * en, 1e-12);
            if constexpr (sizeof(R) == 4) reinterpret_cast<float*>(a.metric)[(a.b0 + b) * a.n_off + off] = (float)v;
            else reinterpret_cast<double*>(a.metric)[(a.b0 + b) * a.n_off + off] = v;
        }
    }
}

// First argmax of each row (np.argmax: the first maximal element; a NaN wins at its first
// occurrence, as numpy's does).  One wave per row.
template <class R>
__global__ __launch_bounds__(ZWG) void row_argmax_kernel(const R* __restrict__ v, int64_t B, int64_t n,
                                                        int64_t* __restrict__ idx, double* __restrict__ val) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * (ZWG / 64) + (threadIdx.x >> 6);
    if (b >= B) return;
    const R* row = v + b * n;
    double best = -INFINITY;
    int64_t bi = n;                                     // sentinel: nothing seen
    bool nan_seen = false;
    for (int64_t j = lane; j < n; j += 64) {
        const double x = (double)row[j];
        if (x != x) { if (!nan_seen) { nan_seen = true; best = x; bi = j; } }
        else if (!nan_seen && (x > best || bi == n)) { best = x; bi = j; }
    }
    // combine: a NaN beats any number (earliest NaN), otherwise larger value, then smaller index
    for (int m = 32; m >= 1; m >>= 1) {
        const double ob = __shfl_xor(best, m);
        const int64_t oi = __shfl_xor(bi, m);
        const bool on = __shfl_xor((int)nan_seen, m) != 0;
        bool take;
        if (oi == n) take = false;
        else if (bi == n) take = true;
        else if (on != nan_seen) take = on;
        else if (on) take = oi < bi;
        else take = (ob > best) || (ob == best && oi < bi);
        if (take) { best = ob; bi = oi; nan_seen = on; }
    }
    if (lane == 0) {
        if (idx) idx[b] = bi == n ? 0 : bi;
        if (val) val[b] = best;
    }
}

// Short rows (n <= 32, e.g. one offset per sequence on cfg5): one thread per row, same semantics.
template <class R>
__global__ __launch_bounds__(ZWG) void row_argmax_short_kernel(const R* __restrict__ v, int64_t B, int32_t n,
                                                              int64_t* __restrict__ idx, double* __restrict__ val) {
    const int64_t b = (int64_t)blockIdx.x * ZWG + threadIdx.x;
    if (b >= B) return;
    const R* row = v + b * n;
    double best = (double)row[0];
    int64_t bi = 0;
    for (int j = 1; j < n && best == best; ++j) {       // stop at the first NaN (it wins)
        const double x = (double)row[j];
        if (x != x || x > best) { best = x; bi = j; }
    }
    if (idx) idx[b] = bi;
    if (val) val[b] = best;
}

template <class R>
void launch_argmax(const R* v, int64_t B, int64_t n, int64_t* idx, double* val, hipStream_t st) {
    if (n <= 32)
        hipLaunchKernelGGL(row_argmax_short_kernel<R>, dim3((unsigned)((B + ZWG - 1) / ZWG)), dim3(ZWG), 0, st, v, B,
                           (int32_t)n, idx, val);
    else
        hipLaunchKernelGGL(row_argmax_kernel<R>, dim3((unsigned)((B + ZWG / 64 - 1) / (ZWG / 64))), dim3(ZWG), 0, st,
                           v, B, n, idx, val);
}

std::once_flag g_setup;

}  // namespace

extern "C" {

int32_t ofs_zc_fft_plan_create3(int32_t precision, int32_t N, int64_t n_windows, int64_t in_dist,
                                int32_t prune_bins, int64_t chunk_windows, void** plan_out, size_t* work_bytes);

int32_t ofs_zc_fft_plan_create(int32_t precision, int32_t N, int64_t n_windows, int64_t in_dist,
                               void** plan_out, size_t* work_bytes) {
    return ofs_zc_fft_plan_create3(precision, N, n_windows, in_dist, 0, 0, plan_out, work_bytes);
}

int32_t ofs_zc_fft_plan_create2(int32_t precision, int32_t N, int64_t n_windows, int64_t in_dist,
                                int32_t prune_bins, void** plan_out, size_t* work_bytes) {
    return ofs_zc_fft_plan_create3(precision, N, n_windows, in_dist, prune_bins, 0, plan_out, work_bytes);
}

static rocfft_status make_fft_plan(int32_t precision, int32_t N, int64_t count, int64_t in_dist, rocfft_plan* out) {
    rocfft_plan_description desc = nullptr;
    if (rocfft_plan_description_create(&desc) != rocfft_status_success) return rocfft_status_failure;
    const size_t len = (size_t)N, stride = 1;
    rocfft_status s = rocfft_plan_description_set_data_layout(
        desc, rocfft_array_type_complex_interleaved, rocfft_array_type_complex_interleaved, nullptr, nullptr,
        1, &stride, (size_t)in_dist, 1, &stride, (size_t)N);
    if (s == rocfft_status_success)
        s = rocfft_plan_create(out, rocfft_placement_notinplace, rocfft_transform_type_complex_forward,
                               precision == OFS_FP32 ? rocfft_precision_single : rocfft_precision_double, 1, &len,
                               (size_t)count, desc);
    rocfft_plan_description_destroy(desc);
    return s;
}

int32_t ofs_zc_fft_plan_create3(int32_t precision, int32_t N, int64_t n_windows, int64_t in_dist,
                                int32_t prune_bins, int64_t chunk_windows, void** plan_out, size_t* work_bytes) {
    if (!plan_out || (precision != OFS_FP32 && precision != OFS_FP64) || N < 1 || n_windows < 1 ||
        in_dist < N || prune_bins < 0 || prune_bins > ZB || chunk_windows < 0 ||
        (prune_bins > 0 && (N > 4096 || (N & (N - 1)))))
        return OFS_EINVAL;
    *plan_out = nullptr;
    std::call_once(g_setup, [] { rocfft_setup(); });
    ZcFftPlan* p = new ZcFftPlan;
    p->chunk = (chunk_windows == 0 || chunk_windows > n_windows) ? n_windows : chunk_windows;
    rocfft_status s = make_fft_plan(precision, N, p->chunk, in_dist, &p->plan);
    if (s == rocfft_status_success && n_windows % p->chunk)
        s = make_fft_plan(precision, N, n_windows % p->chunk, in_dist, &p->tail);
    size_t wb = 0;
    if (s == rocfft_status_success) s = rocfft_plan_get_work_buffer_size(p->plan, &p->work_bytes);
    if (s == rocfft_status_success && p->tail) s = rocfft_plan_get_work_buffer_size(p->tail, &wb);
    if (s != rocfft_status_success) {
        if (p->plan) rocfft_plan_destroy(p->plan);
        if (p->tail) rocfft_plan_destroy(p->tail);
        delete p;
        return OFS_EFFT;
    }
    if (wb > p->work_bytes) p->work_bytes = wb;
    p->precision = precision;
    p->N = N;
    p->n_windows = n_windows;
    p->in_dist = in_dist;
    if (prune_bins > 0) {
        p->prune = prune_bins;
        bool ok = hipMalloc(&p->cb_dev, sizeof(ZcCbData)) == hipSuccess &&
                  hipHostMalloc(&p->cb_host, sizeof(ZcCbData)) == hipSuccess &&
                  (memset(p->cb_host, 0, sizeof(ZcCbData)), true) &&
                  hipMemcpyFromSymbol(&p->cb_fn, precision == OFS_FP32 ? HIP_SYMBOL(zc_store_cb_f32_ptr)
                                                                      : HIP_SYMBOL(zc_store_cb_f64_ptr),
                                      sizeof(void*)) == hipSuccess && p->cb_fn;
        if (!ok) {
            if (p->cb_dev) (void)hipFree(p->cb_dev);
            if (p->cb_host) (void)hipHostFree(p->cb_host);
            rocfft_plan_destroy(p->plan);
            if (p->tail) rocfft_plan_destroy(p->tail);
            delete p;
            return OFS_EHIP;
        }
    }
    if (work_bytes) *work_bytes = p->work_bytes;
    *plan_out = p;
    return OFS_OK;
}

int32_t ofs_zc_fft_plan_create_rows(int32_t precision, int32_t N, int32_t cp, int64_t T, int64_t total_rows,
                                    int64_t rows_per_exec, int32_t prune_bins, void** plan_out, size_t* work_bytes) {
    // prune_bins 0: a DENSE rows plan - no store callback, every window's N-point spectrum written to the
    // caller's [chunk][N] buffer and gathered from there (rocFFT's callback path blocks the host per
    // execution on a synchronous hipMemcpyFromSymbol)
    if (!plan_out || (precision != OFS_FP32 && precision != OFS_FP64) || N < 1 || cp < 0 || total_rows < 1 ||
        rows_per_exec < 0 || prune_bins < 0 || prune_bins > ZB || N > 4096 || (N & (N - 1)))
        return OFS_EINVAL;
    if (T < (int64_t)N + cp) return OFS_ESHORT;
    *plan_out = nullptr;
    std::call_once(g_setup, [] { rocfft_setup(); });
    ZcFftPlan* p = new ZcFftPlan;
    p->rows = (rows_per_exec == 0 || rows_per_exec > total_rows) ? total_rows : rows_per_exec;
    p->row_T = T;
    p->n_off = T - ((int64_t)N + cp) + 1;
    p->cp = cp;
    auto wins = [&](int64_t r) { return (r - 1) * T + p->n_off; };  // windows covering r rows' offsets
    p->chunk = wins(p->rows);
    rocfft_status s = make_fft_plan(precision, N, p->chunk, 1, &p->plan);
    if (s == rocfft_status_success && total_rows % p->rows)
        s = make_fft_plan(precision, N, wins(total_rows % p->rows), 1, &p->tail);
    size_t wb = 0;
    if (s == rocfft_status_success) s = rocfft_plan_get_work_buffer_size(p->plan, &p->work_bytes);
    if (s == rocfft_status_success && p->tail) s = rocfft_plan_get_work_buffer_size(p->tail, &wb);
    if (s != rocfft_status_success) {
        if (p->plan) rocfft_plan_destroy(p->plan);
        if (p->tail) rocfft_plan_destroy(p->tail);
        delete p;
        return OFS_EFFT;
    }
    if (wb > p->work_bytes) p->work_bytes = wb;
    p->precision = precision;
    p->N = N;
    p->n_windows = total_rows;
    p->in_dist = T;
    p->prune = prune_bins;
    bool ok = prune_bins == 0 ||
              (hipMalloc(&p->cb_dev, sizeof(ZcCbData)) == hipSuccess &&
               hipHostMalloc(&p->cb_host, sizeof(ZcCbData)) == hipSuccess &&
               (memset(p->cb_host, 0, sizeof(ZcCbData)), true) &&
               hipMemcpyFromSymbol(&p->cb_fn, precision == OFS_FP32 ? HIP_SYMBOL(zc_store_cb_f32_ptr)
                                                                   : HIP_SYMBOL(zc_store_cb_f64_ptr),
                                   sizeof(void*)) == hipSuccess && p->cb_fn);
    if (!ok) {
        if (p->cb_dev) (void)hipFree(p->cb_dev);
        if (p->cb_host) (void)hipHostFree(p->cb_host);
        rocfft_plan_destroy(p->plan);
        if (p->tail) rocfft_plan_destroy(p->tail);
        delete p;
        return OFS_EHIP;
    }
    if (work_bytes) *work_bytes = p->work_bytes;
    *plan_out = p;
    return OFS_OK;
}

int64_t ofs_zc_fft_plan_chunk(const void* plan) {
    const ZcFftPlan* p = static_cast<const ZcFftPlan*>(plan);
    return p ? p->chunk : 0;
}

int32_t ofs_zc_fft_plan_destroy(void* plan) {
    ZcFftPlan* p = static_cast<ZcFftPlan*>(plan);
    if (!p) return OFS_OK;
    if (p->plan) rocfft_plan_destroy(p->plan);
    if (p->tail) rocfft_plan_destroy(p->tail);
    if (p->cb_dev) (void)hipFree(p->cb_dev);
    if (p->cb_host) (void)hipHostFree(p->cb_host);
    delete p;
    return OFS_OK;
}

int32_t ofs_zc_freq_metric_fft(void* plan, int32_t in_fmt, const void* x, int64_t B, int32_t n_br, int64_t T,
                               int32_t N, int32_t cp, int32_t n_bins, const int32_t* bin_indices,
                               const double* template_bins, double template_energy, void* spectrum, void* work,
                               void* metric, int64_t* peak_index, double* peak_value, void* stream) {
    ZcFftPlan* p = static_cast<ZcFftPlan*>(plan);
    if (!p || !x || !spectrum || !metric || !bin_indices || !template_bins || B < 0 || n_br < 1 || T < 0 ||
        N < 1 || cp < 0 || n_bins < 1 || n_bins > ZB)
        return OFS_EINVAL;
    const int32_t want_fmt = p->precision == OFS_FP32 ? OFS_C64 : OFS_C128;
    if (in_fmt != want_fmt || p->N != N || p->in_dist != T || p->n_windows != B * (int64_t)n_br) return OFS_EINVAL;
    if (p->rows && (p->cp != cp || p->rows % n_br)) return OFS_EINVAL;
    if (p->work_bytes && !work) return OFS_EINVAL;
    if (p->prune && p->prune != n_bins) return OFS_EINVAL;
    if (T < (int64_t)N + cp) return OFS_ESHORT;
    if (B == 0) return OFS_OK;
    const int64_t n_off = T - ((int64_t)N + cp) + 1;
    hipStream_t st = static_cast<hipStream_t>(stream);

    GatherArgs g{};
    g.spec = spectrum;
    g.B = B;
    g.n_off = n_off;
    g.n_br = n_br;
    g.N = p->prune ? n_bins : N;                    // pruned: compact [window][n_bins] rows
    g.n_bins = n_bins;
    g.e_t = template_energy;
    g.metric = metric;
    const int64_t dc = N / 2;
    for (int k = 0; k < n_bins; ++k) {
        const int64_t pos = (((dc + bin_indices[k]) % N) + N) % N;          // zc_freq.py:80
        g.pos[k] = (int32_t)((((pos - N / 2) % N) + N) % N);               // undo fftshift
        g.t_re[k] = template_bins[2 * k];
        g.t_im[k] = template_bins[2 * k + 1];
    }
    if (p->prune) {
        ZcCbData h{};
        h.compact = spectrum;
        h.n_bins = n_bins;
        h.row_T = p->rows ? T : 0;
        h.n_off = p->rows ? n_off : 0;
        while ((1 << h.log2N) < N) ++h.log2N;
        for (int k = 0; k < 4096; ++k) h.slot[k] = -1;
        for (int k = 0; k < n_bins; ++k) {
            if (h.slot[g.pos[k]] >= 0) return OFS_EINVAL;             // duplicate bins: not prunable
            h.slot[g.pos[k]] = (int16_t)k;
            g.pos[k] = k;
        }
        // upload only when the table or the output buffer changed (steady state: no host sync)
        if (memcmp(&h, p->cb_host, sizeof(ZcCbData)) != 0) {
            if (hipStreamSynchronize(st) != hipSuccess) return OFS_EHIP;   // staging may feed a copy
            memcpy(p->cb_host, &h, sizeof(ZcCbData));
            if (hipMemcpyAsync(p->cb_dev, p->cb_host, sizeof(ZcCbData), hipMemcpyHostToDevice, st) != hipSuccess)
                return OFS_EHIP;
        }
    }

    rocfft_execution_info info = nullptr;
    if (rocfft_execution_info_create(&info) != rocfft_status_success) return OFS_EFFT;
    rocfft_status s = rocfft_execution_info_set_stream(info, st);
    if (s == rocfft_status_success && p->work_bytes)
        s = rocfft_execution_info_set_work_buffer(info, work, p->work_bytes);
    if (s == rocfft_status_success && p->prune) {
        void* fns[1] = {p->cb_fn};
        void* dat[1] = {p->cb_dev};
        s = rocfft_execution_info_set_store_callback(info, fns, dat, 0);
    }
    const size_t esz = p->precision == OFS_FP32 ? 8 : 16;
    int32_t rc = OFS_OK;
    if (p->rows) {
        // rows plan: ONE execution per `rows` rows covers every offset of them (windows at distance one
        // sample, the ones straddling two rows dropped by the callback), then one gather over
        // (stream, offset): 2 launches per row group instead of 2 per offset
        const int64_t total = B * (int64_t)n_br;
        for (int64_t r0 = 0; r0 < total && s == rocfft_status_success && rc == OFS_OK; r0 += p->rows) {
            const int64_t nr = total - r0 < p->rows ? total - r0 : p->rows;
            void* in[1] = {const_cast<char*>(static_cast<const char*>(x)) + ((size_t)r0 * T + (size_t)cp) * esz};
            void* out[1] = {spectrum};
            s = rocfft_execute(nr == p->rows ? p->plan : p->tail, in, out, info);
            if (s != rocfft_status_success) break;
            g.b0 = r0 / n_br;
            g.B = nr / n_br;
            const dim3 gr((unsigned)((n_off + ZWG / 64 - 1) / (ZWG / 64)), (unsigned)(g.B < 65535 ? g.B : 65535));
            if (p->precision == OFS_FP32) hipLaunchKernelGGL(zc_gather_rows_kernel<float>, gr, dim3(ZWG), 0, st, g, T);
            else hipLaunchKernelGGL(zc_gather_rows_kernel<double>, gr, dim3(ZWG), 0, st, g, T);
            if (hipGetLastError() != hipSuccess) rc = OFS_EHIP;
        }
    }
    if (p->rows || p->chunk % n_br) {
        rocfft_execution_info_destroy(info);
        if (!p->rows) return OFS_EINVAL;
        if (s != rocfft_status_success) return OFS_EFFT;
        if (rc) return rc;
        if (peak_index || peak_value) {
            if (p->precision == OFS_FP32)
                launch_argmax(static_cast<const float*>(metric), B, n_off, peak_index, peak_value, st);
            else
                launch_argmax(static_cast<const double*>(metric), B, n_off, peak_index, peak_value, st);
            if (hipGetLastError() != hipSuccess) return OFS_EHIP;
        }
        return OFS_OK;
    }
    const int64_t cs = p->chunk / n_br;             // streams per rocFFT execution
    // windows x[b][br][off+cp : off+cp+N], distance T: one batched transform per chunk of streams
    // and offset.  A chunked plan reuses one [chunk][N] spectrum buffer small enough to stay in the
    // Infinity Cache between the FFT's store and the gather's read, and walks a chunk's offsets
    // back to back so its input windows are re-read from cache too.
    for (int64_t b0 = 0; b0 < B && s == rocfft_status_success && rc == OFS_OK; b0 += cs) {
        const int64_t nb = B - b0 < cs ? B - b0 : cs;
        const unsigned gc = (unsigned)((nb + ZWG / 64 - 1) / (ZWG / 64));
        g.b0 = b0;
        g.B = nb;
        for (int64_t off = 0; off < n_off; ++off) {
            void* in[1] = {const_cast<char*>(static_cast<const char*>(x)) +
                           ((size_t)b0 * n_br * T + (size_t)(off + cp)) * esz};
            void* out[1] = {spectrum};
            s = rocfft_execute(nb == cs ? p->plan : p->tail, in, out, info);
            if (s != rocfft_status_success) break;
            g.off = off;
            if (p->precision == OFS_FP32) hipLaunchKernelGGL(zc_gather_kernel<float>, dim3(gc), dim3(ZWG), 0, st, g);
            else hipLaunchKernelGGL(zc_gather_kernel<double>, dim3(gc), dim3(ZWG), 0, st, g);
            if (hipGetLastError() != hipSuccess) { rc = OFS_EHIP; break; }
        }
    }
    rocfft_execution_info_destroy(info);
    if (s != rocfft_status_success) return OFS_EFFT;
    if (rc) return rc;
    if (peak_index || peak_value) {
        if (p->precision == OFS_FP32)
            launch_argmax(static_cast<const float*>(metric), B, n_off, peak_index, peak_value, st);
        else
            launch_argmax(static_cast<const double*>(metric), B, n_off, peak_index, peak_value, st);
        if (hipGetLastError() != hipSuccess) return OFS_EHIP;
    }
    return OFS_OK;
}

int32_t ofs_row_argmax(int32_t precision, const void* v, int64_t B, int64_t n, int64_t* index, double* value,
                       void* stream) {
    if ((precision != OFS_FP32 && precision != OFS_FP64) || !v || B < 0 || n < 1 || (!index && !value))
        return OFS_EINVAL;
    if (B == 0) return OFS_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (precision == OFS_FP32) launch_argmax(static_cast<const float*>(v), B, n, index, value, st);
    else launch_argmax(static_cast<const double*>(v), B, n, index, value, st);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

}  // extern "C"
