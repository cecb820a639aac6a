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

// ------------------------------------------------------------------------------------------
// Frame synthesis: the full per-stream chain of sync_aa.run_single_test (sync_aa.py:699-738),
// every stream its own frame:
//   frame  = [pre_pad zeros][preamble][n_sym random-QPSK OFDM symbols + CP][post_pad zeros]
//            (sync_aa.py:702-712; symbols as build_random_qpsk_symbol, :238-260)
//   y_br   = frame ⊛ cir_br                        (apply_channel_multi_antenna, :577-634)
//   rx_br  = (y_br + CN(0, mean|y_br|^2 / 10^(snr/10))) · exp(i 2π cfo n / fs)   (:625-631, :637-645)
//   out    = quantize_adc(rx, full_scale = rms(rx over all branches) · ratio)  (:263-291, :726-735)
// then the window [win_start + off_b, + T) of every branch.  The preamble part of y is shared
// (preconv = preamble ⊛ cir, host); the QPSK payload is drawn per stream (Philox), inverse-FFT'd
// in LDS (fp64 radix-2) and convolved directly (taps wave-uniform: scalar loads, payload in LDS).
// Two passes: (1) the whole frame, for the per-branch signal power (noise level) and the ADC
// full scale - the noisy power follows from Σ|y|², Σ Re(y·conj g), Σ|g|² without storing rx;
// (2) the window, recomputed and written.
// ------------------------------------------------------------------------------------------
struct FrameArgs {
    const double2* preconv; int64_t Lpc; const double2* cir; int64_t taps; int nb;
    int pre_pad, pre_len, n_sym, n_fft, cp; const int32_t* bins; int n_bins; int post_pad;
    int64_t B, T, win_start; int max_off;
    double snr_lo, snr_hi, cfo_lo, cfo_hi, fs, fs_ratio; uint64_t seed; int fmt;
    void* out; double* params; uint8_t* phases;
};
constexpr int FW = 256;
constexpr int FNB = 4;                 // branches supported

__device__ __forceinline__ int brev(int v, int bits) { return (int)(__brev((unsigned)v) >> (32 - bits)); }

// noise pair of (stream, branch, sample): Box-Muller on a Philox draw
__device__ __forceinline__ double2 gauss(int64_t n, int br, int64_t b, uint32_t k0, uint32_t k1) {
    const u4 r = philox(u4{(uint32_t)n, (uint32_t)(n >> 32), (uint32_t)br | 0x40000000u, (uint32_t)b}, k0, k1);
    const double rad = sqrt(-2.0 * log(u01(r.x, r.y)));
    double gs, gc;
    sincospi(2.0 * u01(r.z, r.w), &gs, &gc);
    return make_double2(rad * gc, rad * gs);
}

// y_br[n] of the noiseless frame: shared preamble part + this stream's payload part
__device__ __forceinline__ double2 frame_y(const FrameArgs& a, const double2* pay, int64_t Lp, int br, int64_t n) {
    double yr = 0.0, yi = 0.0;
    const int64_t q0 = n - a.pre_pad;
    if (q0 >= 0 && q0 < a.Lpc) { const double2 v = a.preconv[br * a.Lpc + q0]; yr = v.x; yi = v.y; }
    const int64_t p0 = (int64_t)a.pre_pad + a.pre_len;
    const int64_t jlo = max((int64_t)0, n - p0 - Lp + 1), jhi = min(a.taps - 1, n - p0);
    const double2* h = a.cir + br * a.taps;
    for (int64_t j = jlo; j <= jhi; ++j) {
        const double2 hv = h[j], pv = pay[n - p0 - j];
        yr = fma(hv.x, pv.x, fma(-hv.y, pv.y, yr));
        yi = fma(hv.x, pv.y, fma(hv.y, pv.x, yi));
    }
    return make_double2(yr, yi);
}

__global__ __launch_bounds__(FW) void synth_frames_kernel(FrameArgs a) {
    extern __shared__ double2 fsm[];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = a.n_fft, S = a.n_fft + a.cp, lb = 31 - __clz(N);
    const int64_t Lp = (int64_t)a.n_sym * S;
    double2* pay = fsm;                            // [n_sym][N + cp]
    double2* buf = pay + Lp;                       // [N]
    double2* tw = buf + N;                         // [N / 2]: exp(+2πi j / N)
    double* red = reinterpret_cast<double*>(tw + N / 2);   // [FW / 64][FNB][3] block reduction
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32) ^ (uint32_t)b * 0x85EBCA6Bu;
    const u4 d = philox(u4{(uint32_t)b, (uint32_t)(b >> 32), 0xFFFFFFFFu, 0xFFFFFFFFu}, k0, k1);
    const int off = a.max_off > 1 ? (int)(u01(d.x, d.y) * a.max_off - 1e-9) : 0;
    const double snr = a.snr_lo + (a.snr_hi - a.snr_lo) * u01(d.z, d.w);
    const u4 d2 = philox(u4{(uint32_t)b, (uint32_t)(b >> 32), 0xFFFFFFFEu, 0xFFFFFFFFu}, k0, k1);
    const double cfo = a.cfo_lo + (a.cfo_hi - a.cfo_lo) * u01(d2.x, d2.y);

    for (int j = tid; j < N / 2; j += FW) {
        double s_, c_;
        sincospi(2.0 * (double)j / (double)N, &s_, &c_);
        tw[j] = make_double2(c_, s_);
    }
    // ---- payload: n_sym random-QPSK symbols, inverse FFT (DIT, bit-reversed load), CP ----
    const double qs = 0.70710678118654752440;      // 1/sqrt(2)
    const double norm = 1.0 / sqrt(0.5 * (double)a.n_bins);   // unit mean power (Parseval)
    for (int s = 0; s < a.n_sym; ++s) {
        for (int j = tid; j < N; j += FW) buf[j] = make_double2(0.0, 0.0);
        __syncthreads();
        for (int i = tid; i < a.n_bins; i += FW) {
            const u4 r = philox(u4{(uint32_t)i, (uint32_t)s, 0x7FFFFFFFu, (uint32_t)b}, k0, k1);
            const int ph = (int)(r.x & 3u);
            double sn, cs;
            sincospi(0.25 * (double)(2 * ph + 1), &sn, &cs);
            buf[brev(a.bins[i], lb)] = make_double2(cs * qs, sn * qs);
            if (a.phases) a.phases[(b * a.n_sym + s) * a.n_bins + i] = (uint8_t)ph;
        }
        __syncthreads();
        for (int len = 2; len <= N; len <<= 1) {
            const int half = len >> 1, step = N / len;
            for (int j = tid; j < N / 2; j += FW) {
                const int g = j / half, k = j - g * half;
                const int p = g * len + k, q = p + half;
                const double2 w = tw[k * step], v = buf[q];
                const double2 t = make_double2(w.x * v.x - w.y * v.y, w.x * v.y + w.y * v.x);
                const double2 u = buf[p];
                buf[p] = make_double2(u.x + t.x, u.y + t.y);
                buf[q] = make_double2(u.x - t.x, u.y - t.y);
            }
            __syncthreads();
        }
        for (int n = tid; n < N; n += FW) {
            const double2 v = make_double2(buf[n].x * norm, buf[n].y * norm);
            pay[(int64_t)s * S + a.cp + n] = v;
            if (n >= N - a.cp) pay[(int64_t)s * S + n - (N - a.cp)] = v;
        }
        __syncthreads();
    }
    // ---- pass 1: whole-frame statistics per branch ----
    const int64_t Lf = (int64_t)a.pre_pad + a.pre_len + Lp + a.post_pad;
    const int64_t Lout = Lf + a.taps - 1;
    double syy[FNB], syg[FNB], sgg[FNB];
#pragma unroll
    for (int br = 0; br < FNB; ++br) { syy[br] = 0.0; syg[br] = 0.0; sgg[br] = 0.0; }
    for (int br = 0; br < a.nb; ++br)
        for (int64_t n = tid; n < Lout; n += FW) {
            const double2 y = frame_y(a, pay, Lp, br, n);
            const double2 g = gauss(n, br, b, k0, k1);
            syy[br] += y.x * y.x + y.y * y.y;
            syg[br] += y.x * g.x + y.y * g.y;
            sgg[br] += g.x * g.x + g.y * g.y;
        }
    const int w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int br = 0; br < FNB; ++br) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            syy[br] += __shfl_xor(syy[br], o, 64); syg[br] += __shfl_xor(syg[br], o, 64);
            sgg[br] += __shfl_xor(sgg[br], o, 64);
        }
        if (lane == 0) { red[(w * FNB + br) * 3] = syy[br]; red[(w * FNB + br) * 3 + 1] = syg[br]; red[(w * FNB + br) * 3 + 2] = sgg[br]; }
    }
    __syncthreads();
    double sd[FNB], p_all = 0.0;
    const double snr_lin = pow(10.0, snr / 10.0);
#pragma unroll
    for (int br = 0; br < FNB; ++br) {
        double Y = 0.0, YG = 0.0, GG = 0.0;
        for (int q = 0; q < FW / 64; ++q) { Y += red[(q * FNB + br) * 3]; YG += red[(q * FNB + br) * 3 + 1]; GG += red[(q * FNB + br) * 3 + 2]; }
        sd[br] = br < a.nb ? sqrt(Y / (double)Lout / snr_lin / 2.0) : 0.0;          // channel.py-style noise std
        if (br < a.nb) p_all += Y + 2.0 * sd[br] * YG + sd[br] * sd[br] * GG;       // Σ|y + sd g|² (tone: |.| = 1)
    }
    const double full_scale = sqrt(p_all / ((double)a.nb * (double)Lout)) * a.fs_ratio;
    if (a.params && tid == 0) {
        a.params[4 * b] = (double)(a.win_start + off); a.params[4 * b + 1] = snr; a.params[4 * b + 2] = cfo;
        a.params[4 * b + 3] = a.fs_ratio > 0.0 ? full_scale : 0.0;
    }
    // ---- pass 2: the window ----
    const double wc = 2.0 * M_PI * cfo / a.fs;
    const double levels = 2048.0;
    for (int br = 0; br < a.nb; ++br)
        for (int64_t t = tid; t < a.T; t += FW) {
            const int64_t n = a.win_start + off + t;
            double re = 0.0, im = 0.0;
            if (n >= 0 && n < Lout) {
                const double2 y = frame_y(a, pay, Lp, br, n);
                const double2 g = gauss(n, br, b, k0, k1);
                const double xr = y.x + sd[br] * g.x, xi = y.y + sd[br] * g.y;
                double sn, cs;
                sincos(wc * (double)n, &sn, &cs);
                re = xr * cs - xi * sn;
                im = xr * sn + xi * cs;
            }
            const int64_t o = (b * a.nb + br) * a.T + t;
            if (a.fs_ratio > 0.0) {                                   // quantize_adc (sync_aa.py:263-291)
                const double cr = rint(fmin(fmax(re / full_scale, -1.0), 1.0 - 1.0 / levels) * levels);
                const double ci = rint(fmin(fmax(im / full_scale, -1.0), 1.0 - 1.0 / levels) * levels);
                if (a.fmt == OFS_CI16) {
                    static_cast<short2*>(a.out)[o] = make_short2((short)cr, (short)ci);
                    continue;
                }
                re = cr / levels * full_scale;
                im = ci / levels * full_scale;
            }
            if (a.fmt == OFS_C64) static_cast<float2*>(a.out)[o] = make_float2((float)re, (float)im);
            else if (a.fmt == OFS_C128) static_cast<double2*>(a.out)[o] = make_double2(re, im);
            else static_cast<short2*>(a.out)[o] = make_short2((short)fmin(fmax(rint(re), -32768.0), 32767.0),
                                                             (short)fmin(fmax(rint(im), -32768.0), 32767.0));
        }
}

}  // namespace

extern "C" int32_t ofs_synth_frames(const void* preconv, int64_t preconv_len, const void* cir, int64_t taps,
                                    int32_t n_br, int32_t pre_pad, int32_t pre_len, int32_t n_sym, int32_t n_fft,
                                    int32_t cp_len, const int32_t* bins, int32_t n_bins, int32_t post_pad, int64_t B,
                                    int64_t T, int64_t win_start, int32_t max_offset, double snr_lo_db,
                                    double snr_hi_db, double cfo_lo_hz, double cfo_hi_hz, double fs_hz,
                                    double full_scale_ratio, uint64_t seed, int32_t out_fmt, void* out,
                                    double* params, uint8_t* phases, void* stream) {
    if (!preconv || !cir || !out || preconv_len < 1 || taps < 1 || n_br < 1 || n_br > FNB || pre_pad < 0 ||
        pre_len < 0 || n_sym < 0 || cp_len < 0 || post_pad < 0 || B < 0 || T < 0 || max_offset < 0 ||
        !(fs_hz > 0.0) || B > 0x7fffffff || n_fft < 2 || n_fft > 4096 || (n_fft & (n_fft - 1)) || cp_len > n_fft ||
        (n_sym > 0 && (!bins || n_bins < 1 || n_bins > n_fft)) || preconv_len != (int64_t)pre_len + taps - 1 ||
        !(out_fmt == OFS_C64 || out_fmt == OFS_C128 || out_fmt == OFS_CI16))
        return OFS_EINVAL;
    if (B == 0 || T == 0) return OFS_OK;
    const size_t lds = ((size_t)n_sym * (n_fft + cp_len) + n_fft + n_fft / 2) * sizeof(double2) +
                       (size_t)(FW / 64) * FNB * 3 * sizeof(double);
    if (lds > 160 * 1024) return OFS_ETOOLONG;
    FrameArgs a{static_cast<const double2*>(preconv), preconv_len, static_cast<const double2*>(cir), taps, n_br,
                pre_pad, pre_len, n_sym, n_fft, cp_len, bins, n_bins, post_pad, B, T, win_start, max_offset,
                snr_lo_db, snr_hi_db, cfo_lo_hz, cfo_hi_hz, fs_hz, full_scale_ratio, seed, out_fmt, out, params,
                phases};
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void*)synth_frames_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
        return OFS_EHIP;
    hipLaunchKernelGGL(synth_frames_kernel, dim3((unsigned)B), dim3(FW), lds, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? OFS_OK : OFS_EHIP;
}

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
