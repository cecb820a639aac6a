// synth.hip — batched receive-stream synthesis on the GPU: the channel +
// impairment chain of the reference's drivers (channel.apply_channel, channel.py:80-98;
// core.apply_cfo, core.py:123-138; sync_aa.apply_channel_multi_antenna / quantize_adc,
// sync_aa.py:263-291, :577-645) restated for benchmark-scale batches:
//
//   out[b][br][n] = q( base[br][off_b + n] · exp(i 2π cfo_b n / fs) + w[b][br][n] ),
//   off_b ~ U{0 .. max_offset-1},  snr_b ~ U[snr_lo, snr_hi] dB,  cfo_b ~ U[cfo_lo, cfo_hi] Hz,
//   w ~ CN(0, 10^(-snr_b/10))  (unit-power base),  q = none | int12 ADC (round, clip ±2047).
//
// `base` is the faded preamble per branch (preamble ⊛ CIR, built once on the host): the
// per-stream work is a shifted read, a tone and noise - memory-bound, one pass over the output.
// Randomness: Philox-4x32-10 keyed by (seed, stream) with the sample index as counter, Box-Muller
// for the Gaussian pairs.  Deterministic for a seed; distribution-level parity only (the
// reference draws from numpy's PCG64, which the task does not require to reproduce).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "ofdmsync.h"

namespace {

struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = u4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return c;
}
// uniform in (0, 1]
__device__ __forceinline__ double u01(uint32_t a, uint32_t b) {
    const uint64_t v = ((uint64_t)(a >> 5) << 26) | (b >> 6);          // 53 bits
    return ((double)v + 1.0) * (1.0 / 9007199254740992.0);
}

struct SynArgs {
    const double2* base; int64_t Lb; int64_t B, T; int nb; int max_off;
    double snr_lo, snr_hi, cfo_lo, cfo_hi, fs; uint64_t seed; int fmt; double adc_scale;
    void* out; double* params;
};

constexpr int SW = 256;

__global__ __launch_bounds__(SW) void synth_kernel(SynArgs a) {
    const int64_t b = blockIdx.x;
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32) ^ (uint32_t)b * 0x85EBCA6Bu;
    // per-stream draws: counter (b, ~0) is outside the per-sample counters
    const u4 d = philox(u4{(uint32_t)b, (uint32_t)(b >> 32), 0xFFFFFFFFu, 0xFFFFFFFFu}, k0, k1);
    const int off = a.max_off > 1 ? (int)(u01(d.x, d.y) * a.max_off - 1e-9) : 0;
    const double snr = a.snr_lo + (a.snr_hi - a.snr_lo) * u01(d.z, d.w);
    const u4 d2 = philox(u4{(uint32_t)b, (uint32_t)(b >> 32), 0xFFFFFFFEu, 0xFFFFFFFFu}, k0, k1);
    const double cfo = a.cfo_lo + (a.cfo_hi - a.cfo_lo) * u01(d2.x, d2.y);
    const double sd = sqrt(pow(10.0, -snr / 10.0) / 2.0);
    if (a.params && threadIdx.x == 0) {
        a.params[3 * b] = off; a.params[3 * b + 1] = snr; a.params[3 * b + 2] = cfo;
    }
    const double w = 2.0 * M_PI * cfo / a.fs;
    for (int64_t n = threadIdx.x; n < a.T; n += SW) {
        double sn, cs;
        sincos(w * (double)n, &sn, &cs);
        for (int br = 0; br < a.nb; ++br) {
            const int64_t j = off + n;
            const double2 s = j < a.Lb ? a.base[br * a.Lb + j] : make_double2(0.0, 0.0);
            const u4 r = philox(u4{(uint32_t)n, (uint32_t)(n >> 32), (uint32_t)br, (uint32_t)b}, k0, k1);
            const double rad = sqrt(-2.0 * log(u01(r.x, r.y)));
            double gs, gc;
            sincospi(2.0 * u01(r.z, r.w), &gs, &gc);
            const double re = s.x * cs - s.y * sn + sd * rad * gc;
            const double im = s.x * sn + s.y * cs + sd * rad * gs;
            const int64_t o = (b * a.nb + br) * a.T + n;
            if (a.fmt == OFS_C64) {
                static_cast<float2*>(a.out)[o] = make_float2((float)re, (float)im);
            } else if (a.fmt == OFS_C128) {
                static_cast<double2*>(a.out)[o] = make_double2(re, im);
            } else {
                const double qr = fmin(fmax(rint(re * a.adc_scale), -2048.0), 2047.0);
                const double qi = fmin(fmax(rint(im * a.adc_scale), -2048.0), 2047.0);
                static_cast<short2*>(a.out)[o] = make_short2((short)qr, (short)qi);
            }
        }
    }
}

}  // namespace

extern "C" int32_t ofs_synth_batch(const void* base, int64_t base_len, int32_t n_br, int64_t B, int64_t T,
                                   int32_t max_offset, double snr_lo_db, double snr_hi_db, double cfo_lo_hz,
                                   double cfo_hi_hz, double fs_hz, uint64_t seed, int32_t out_fmt,
                                   double adc_scale, void* out, double* params, void* stream) {
    if (!base || !out || base_len < 1 || n_br < 1 || B < 0 || T < 0 || max_offset < 0 || !(fs_hz > 0.0) ||
        !(out_fmt == OFS_C64 || out_fmt == OFS_C128 || out_fmt == OFS_CI16) || B > 0x7fffffff)
        return OFS_EINVAL;
    if (B == 0 || T == 0) return OFS_OK;
    SynArgs a{static_cast<const double2*>(base), base_len, B, T, n_br, max_offset, snr_lo_db, snr_hi_db,
              cfo_lo_hz, cfo_hi_hz, fs_hz, seed, out_fmt, adc_scale, out, params};
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)B), dim3(SW), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}
