// sol_stream.hip — speed-of-light probe for the headline kernel's memory pattern.
//
// The fused S&C kernel reads 8 B (complex64 x) and writes 16 B (complex64 P, f32 R, f32 M) per
// sample over 65536 streams x 1024 samples.  This program times kernels that move exactly those
// bytes with trivial arithmetic, so the headline's roofline fraction can be read against what
// the chip actually sustains for a 1:2 read:write stream (and against a plain float4 copy,
// the 6.3 TB/s figure of MI355X_MICROARCH.md).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/sol_stream tools/sol_stream.hip
//   tools/bin/sol_stream [B] [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// float4 copy, grid-stride
__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, int64_t n4) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

// the headline pattern, flat: a thread handles 4 consecutive samples
__global__ void pattern_flat(const float4* __restrict__ x, float4* __restrict__ P, float4* __restrict__ R,
                             float4* __restrict__ M, int64_t nq) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
        const float4 a = x[2 * q], c = x[2 * q + 1];
        P[2 * q] = a; P[2 * q + 1] = c;
        const float4 r = make_float4(a.x * a.x + a.y * a.y, a.z * a.z + a.w * a.w, c.x * c.x + c.y * c.y,
                                     c.z * c.z + c.w * c.w);
        R[q] = r;
        M[q] = make_float4(r.x * 0.5f, r.y * 0.5f, r.z * 0.5f, r.w * 0.5f);
    }
}

// the headline pattern, one wave per stream (the aa_fast geometry: 4 waves per 256-thread
// workgroup, lane owns 4 consecutive samples of each 256-sample row); all loads first
template <int T>
__global__ __launch_bounds__(256) void pattern_wave(const float4* __restrict__ x, float4* __restrict__ P,
                                                    float4* __restrict__ R, float4* __restrict__ M, int64_t B) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    constexpr int RW = T / 256;
    float4 v[RW][2];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        const int64_t q = (b * T + 256 * k + 4 * lane) / 2;
        v[k][0] = x[q]; v[k][1] = x[q + 1];
    }
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        const int64_t s = b * T + 256 * k + 4 * lane;
        P[s / 2] = v[k][0]; P[s / 2 + 1] = v[k][1];
        const float4 a = v[k][0], c = v[k][1];
        const float4 r = make_float4(a.x * a.x + a.y * a.y, a.z * a.z + a.w * a.w, c.x * c.x + c.y * c.y,
                                     c.z * c.z + c.w * c.w);
        R[s / 4] = r;
        M[s / 4] = make_float4(r.x * 0.5f, r.y * 0.5f, r.z * 0.5f, r.w * 0.5f);
    }
}

// pattern_wave with one wave (= one stream) per 64-thread workgroup: the round-6 headline geometry,
// launched with unused dynamic LDS to cap the workgroups per CU as the headline does (16 KiB = 10)
template <int T>
__global__ __launch_bounds__(64) void pattern_wave1(const float4* __restrict__ x, float4* __restrict__ P,
                                                   float4* __restrict__ R, float4* __restrict__ M, int64_t B) {
    const int lane = threadIdx.x & 63;
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    constexpr int RW = T / 256;
    float4 v[RW][2];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        const int64_t q = (b * T + 256 * k + 4 * lane) / 2;
        v[k][0] = x[q]; v[k][1] = x[q + 1];
    }
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        const int64_t s = b * T + 256 * k + 4 * lane;
        P[s / 2] = v[k][0]; P[s / 2 + 1] = v[k][1];
        const float4 a = v[k][0], c = v[k][1];
        const float4 r = make_float4(a.x * a.x + a.y * a.y, a.z * a.z + a.w * a.w, c.x * c.x + c.y * c.y,
                                     c.z * c.z + c.w * c.w);
        R[s / 4] = r;
        M[s / 4] = make_float4(r.x * 0.5f, r.y * 0.5f, r.z * 0.5f, r.w * 0.5f);
    }
}

// pattern_wave with the headline kernel's shape of a wave's life: the stream DMA'd into LDS
// (global_load_lds_dwordx4), then per row a dependent VALU chain of NV ops (standing in for the
// metric arithmetic) before the row's stores
template <int T, int NV>
__global__ __launch_bounds__(256) void pattern_lds(const float4* __restrict__ x, float4* __restrict__ P,
                                                   float4* __restrict__ R, float4* __restrict__ M, int64_t B) {
    constexpr int RW = T / 256;
    __shared__ float4 lds[4][RW * 2][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t b = (int64_t)blockIdx.x * 4 + w;
    if (b >= B) return;
    const float2* xs = reinterpret_cast<const float2*>(x) + b * T;
#pragma unroll
    for (int k = 0; k < RW; ++k)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(xs + 256 * k + 4 * lane + 2 * j),
                                             (__attribute__((address_space(3))) void*)&lds[w][k * 2 + j][0], 16, 0, 0);
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        float4 a = lds[w][2 * k][lane], c = lds[w][2 * k + 1][lane];
        float acc = a.x;
#pragma unroll
        for (int i = 0; i < NV; ++i) acc = fmaf(acc, 0.999f, c.y);
        a.x += acc * 1e-30f;
        const int64_t s = b * T + 256 * k + 4 * lane;
        P[s / 2] = a; P[s / 2 + 1] = c;
        const float4 r = make_float4(a.x * a.x + a.y * a.y, a.z * a.z + a.w * a.w, c.x * c.x + c.y * c.y,
                                     c.z * c.z + c.w * c.w);
        R[s / 4] = r;
        M[s / 4] = make_float4(r.x * 0.5f, r.y * 0.5f, r.z * 0.5f, r.w * 0.5f);
    }
}

// the cfg4 pattern (fused combined S&C + Minn, combined_sc_min.py:333-335): 8 B read and two
// output sets of P c64 + R f32 + M f32 = 32 B written per sample (1:4), flat, 16 B per lane
__global__ void pattern_cfg4(const float4* __restrict__ x, float4* __restrict__ P1, float4* __restrict__ R1,
                             float4* __restrict__ M1, float4* __restrict__ P2, float4* __restrict__ R2,
                             float4* __restrict__ M2, int64_t nq) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
        const float4 a = x[2 * q], c = x[2 * q + 1];
        const float4 r = make_float4(a.x * a.x + a.y * a.y, a.z * a.z + a.w * a.w, c.x * c.x + c.y * c.y,
                                     c.z * c.z + c.w * c.w);
        P1[2 * q] = a; P1[2 * q + 1] = c; R1[q] = r; M1[q] = make_float4(r.x * 0.5f, r.y, r.z, r.w);
        P2[2 * q] = c; P2[2 * q + 1] = a; R2[q] = make_float4(r.w, r.z, r.y, r.x);
        M2[q] = make_float4(r.x * 0.25f, r.y, r.z, r.w);
    }
}

// the same 1:4 mix with 8 B per lane (float2) stores at a 4-byte-misaligned base, as the fused
// kernel's [B][T-N+1] output rows force (odd row length, d0 = nb - (N-1))
__global__ void pattern_cfg4_f2(const float4* __restrict__ x, float2* __restrict__ P1, float2* __restrict__ R1,
                                float2* __restrict__ M1, float2* __restrict__ P2, float2* __restrict__ R2,
                                float2* __restrict__ M2, int64_t nh) {
    for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < nh; h += (int64_t)gridDim.x * blockDim.x) {
        const float4 a = x[h];
        const float2 r = make_float2(a.x * a.x + a.y * a.y, a.z * a.z + a.w * a.w);
        float* p1 = reinterpret_cast<float*>(P1) + 1;             // misaligned by one float
        float* r1 = reinterpret_cast<float*>(R1) + 1;
        float* m1 = reinterpret_cast<float*>(M1) + 1;
        float* p2 = reinterpret_cast<float*>(P2) + 1;
        float* r2 = reinterpret_cast<float*>(R2) + 1;
        float* m2 = reinterpret_cast<float*>(M2) + 1;
        typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
        typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
        *reinterpret_cast<f4u*>(p1 + 4 * h) = f4u{a.x, a.y, a.z, a.w};
        *reinterpret_cast<f2u*>(r1 + 2 * h) = f2u{r.x, r.y};
        *reinterpret_cast<f2u*>(m1 + 2 * h) = f2u{r.x * 0.5f, r.y};
        *reinterpret_cast<f4u*>(p2 + 4 * h) = f4u{a.z, a.w, a.x, a.y};
        *reinterpret_cast<f2u*>(r2 + 2 * h) = f2u{r.y, r.x};
        *reinterpret_cast<f2u*>(m2 + 2 * h) = f2u{r.x * 0.25f, r.y};
    }
}

// read-only and write-only streams
__global__ void read4(const float4* __restrict__ a, float* out, int64_t n4) {
    float s = 0.f;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678f) out[0] = s;
}
__global__ void write4(float4* __restrict__ a, int64_t n4) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

// cfg2b (minn_rtl int12) byte mix: 4 B in, six f64 arrays + two u8 arrays out (50 B) per sample;
// a thread handles 2 consecutive samples (16-byte stores per f64 array)
__global__ void pattern_cfg2b(const int2* __restrict__ x, double2* o0, double2* o1, double2* o2, double2* o3,
                              double2* o4, double2* o5, uchar2* f0, uchar2* f1, int64_t n2) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n2; q += (int64_t)gridDim.x * blockDim.x) {
        const int2 w = x[q];
        const double a = (double)w.x, b = (double)w.y;
        o0[q] = make_double2(a, b); o1[q] = make_double2(b, a); o2[q] = make_double2(a + 1, b);
        o3[q] = make_double2(a, b + 1); o4[q] = make_double2(a * 2, b); o5[q] = make_double2(a, b * 2);
        f0[q] = make_uchar2((unsigned char)w.x, (unsigned char)w.y); f1[q] = make_uchar2(1, (unsigned char)q);
    }
}

template <class F>
static double time_ms(F f, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGetLastError());
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
    return ms / iters;
}

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? atoll(argv[1]) : 65536;
    const int64_t T = 1024;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const int64_t n = B * T;
    float4 *x, *P, *R, *M;
    float* dummy;
    CK(hipMalloc(&x, n * 8)); CK(hipMalloc(&P, n * 8)); CK(hipMalloc(&R, n * 4)); CK(hipMalloc(&M, n * 4));
    CK(hipMalloc(&dummy, 64));
    CK(hipMemset(x, 0, n * 8));
    int dev;
    hipDeviceProp_t pr;
    CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&pr, dev));
    const int cus = pr.multiProcessorCount;
    printf("{\"device\": \"%s\", \"cus\": %d, \"B\": %ld, \"T\": %ld}\n", pr.gcnArchName, cus, (long)B, (long)T);
    auto report = [&](const char* name, double bytes, double ms) {
        printf("{\"probe\": \"%s\", \"ms\": %.5f, \"GBs\": %.1f, \"frac_8TBs\": %.4f}\n", name, ms, bytes / ms / 1e6,
               bytes / ms / 1e6 / 8000.0);
    };
    const int64_t n4 = n * 8 / 16;
    char nm[96];
    for (int grid_mult : {4, 8, 16}) {
        const int grid = cus * grid_mult;
        snprintf(nm, sizeof nm, "copy4 grid=%dxCU", grid_mult);
        report(nm, 2.0 * n * 8, time_ms([&] { copy4<<<grid, 256>>>(x, P, n4); }, iters));
        snprintf(nm, sizeof nm, "read4 grid=%dxCU", grid_mult);
        report(nm, 1.0 * n * 8, time_ms([&] { read4<<<grid, 256>>>(x, dummy, n4); }, iters));
        snprintf(nm, sizeof nm, "write4 grid=%dxCU", grid_mult);
        report(nm, 1.0 * n * 8, time_ms([&] { write4<<<grid, 256>>>(P, n4); }, iters));
        snprintf(nm, sizeof nm, "pattern_flat(8r+16w) grid=%dxCU", grid_mult);
        report(nm, 24.0 * n, time_ms([&] { pattern_flat<<<grid, 256>>>(x, P, R, M, n / 4); }, iters));
    }
    report("pattern_flat(8r+16w) grid=full", 24.0 * n,
           time_ms([&] { pattern_flat<<<(unsigned)((n / 4 + 255) / 256), 256>>>(x, P, R, M, n / 4); }, iters));
    report("pattern_wave(8r+16w) wave-per-stream", 24.0 * n,
           time_ms([&] { pattern_wave<1024><<<(unsigned)((B + 3) / 4), 256>>>(x, P, R, M, B); }, iters));
    for (int pad : {0, 13000, 14800, 16384, 18000, 20480}) {
        snprintf(nm, sizeof nm, "pattern_wave1(8r+16w) 64-thread wg, LDS pad %d", pad);
        report(nm, 24.0 * n, time_ms([&] { pattern_wave1<1024><<<(unsigned)B, 64, pad>>>(x, P, R, M, B); }, iters));
    }
    report("pattern_lds<NV=0>", 24.0 * n,
           time_ms([&] { pattern_lds<1024, 0><<<(unsigned)((B + 3) / 4), 256>>>(x, P, R, M, B); }, iters));
    report("pattern_lds<NV=64>", 24.0 * n,
           time_ms([&] { pattern_lds<1024, 64><<<(unsigned)((B + 3) / 4), 256>>>(x, P, R, M, B); }, iters));
    report("pattern_lds<NV=256>", 24.0 * n,
           time_ms([&] { pattern_lds<1024, 256><<<(unsigned)((B + 3) / 4), 256>>>(x, P, R, M, B); }, iters));
    report("pattern_lds<NV=512>", 24.0 * n,
           time_ms([&] { pattern_lds<1024, 512><<<(unsigned)((B + 3) / 4), 256>>>(x, P, R, M, B); }, iters));
    {   // cfg4 mix: 8 B in, 32 B out per sample (same sample count)
        float4 *P2, *R2, *M2;
        CK(hipMalloc(&P2, n * 8 + 64)); CK(hipMalloc(&R2, n * 4 + 64)); CK(hipMalloc(&M2, n * 4 + 64));
        float4 *P1b, *R1b, *M1b;
        CK(hipMalloc(&P1b, n * 8 + 64)); CK(hipMalloc(&R1b, n * 4 + 64)); CK(hipMalloc(&M1b, n * 4 + 64));
        for (int grid_mult : {8, 16}) {
            snprintf(nm, sizeof nm, "pattern_cfg4(8r+32w, 16B stores) grid=%dxCU", grid_mult);
            report(nm, 40.0 * n, time_ms([&] { pattern_cfg4<<<cus * grid_mult, 256>>>(x, P1b, R1b, M1b, P2, R2, M2, n / 4); }, iters));
            snprintf(nm, sizeof nm, "pattern_cfg4_f2(8r+32w, misaligned 8B stores) grid=%dxCU", grid_mult);
            report(nm, 40.0 * n, time_ms([&] { pattern_cfg4_f2<<<cus * grid_mult, 256>>>(x, (float2*)P1b, (float2*)R1b, (float2*)M1b,
                                                                                         (float2*)P2, (float2*)R2, (float2*)M2, n / 2); }, iters));
        }
        report("pattern_cfg4(8r+32w, 16B stores) grid=full", 40.0 * n,
               time_ms([&] { pattern_cfg4<<<(unsigned)((n / 4 + 255) / 256), 256>>>(x, P1b, R1b, M1b, P2, R2, M2, n / 4); }, iters));
        report("pattern_cfg4_f2(8r+32w, misaligned 8B stores) grid=full", 40.0 * n,
               time_ms([&] { pattern_cfg4_f2<<<(unsigned)((n / 2 + 255) / 256), 256>>>(x, (float2*)P1b, (float2*)R1b, (float2*)M1b,
                                                                                         (float2*)P2, (float2*)R2, (float2*)M2, n / 2); }, iters));
        report("write4 grid=full", 1.0 * n * 8,
               time_ms([&] { write4<<<(unsigned)((n * 8 / 16 + 255) / 256), 256>>>(P1b, n * 8 / 16); }, iters));
        CK(hipFree(P2)); CK(hipFree(R2)); CK(hipFree(M2)); CK(hipFree(P1b)); CK(hipFree(R1b)); CK(hipFree(M1b));
    }
    {   // cfg2b mix at this B (4096 = the cfg2b batch): 4 B in, 50 B out per sample
        double2* o[6];
        uchar2 *f0, *f1;
        for (auto& p : o) CK(hipMalloc(&p, n * 8));
        CK(hipMalloc(&f0, n)); CK(hipMalloc(&f1, n));
        for (int grid_mult : {4, 8, 16}) {
            snprintf(nm, sizeof nm, "pattern_cfg2b(4r+50w) grid=%dxCU", grid_mult);
            report(nm, 54.0 * n, time_ms([&] { pattern_cfg2b<<<cus * grid_mult, 256>>>((const int2*)x, o[0], o[1], o[2], o[3],
                                                                                          o[4], o[5], f0, f1, n / 2); }, iters));
        }
        report("pattern_cfg2b(4r+50w) grid=full", 54.0 * n,
               time_ms([&] { pattern_cfg2b<<<(unsigned)((n / 2 + 255) / 256), 256>>>((const int2*)x, o[0], o[1], o[2], o[3],
                                                                                     o[4], o[5], f0, f1, n / 2); }, iters));
        for (auto& p : o) CK(hipFree(p));
        CK(hipFree(f0)); CK(hipFree(f1));
    }
    report("pattern_wave(8r+16w) wave-per-stream again", 24.0 * n,
           time_ms([&] { pattern_wave<1024><<<(unsigned)((B + 3) / 4), 256>>>(x, P, R, M, B); }, iters));
    return 0;
}
