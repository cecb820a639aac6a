// Dependent-chain latency probe (diagnostic): cycles per dependent v_add_f64 / v_add_f32 /
// v_fma_f64 in one wave, measured with s_memtime around a long unrolled chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <class T, int OP>
__global__ void chain(T* out, long long* cyc, T a0, T b0, int iters) {
    T acc = a0 + (T)threadIdx.x, x = b0, y = b0 * (T)0.5;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 64; ++u) {
            if (OP == 0) acc = (acc + x) - y;          // 2 dependent adds
            else acc = acc * x + y;                    // 1 dependent fma
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double* od; float* of; long long* c;
    hipMalloc(&od, 64 * 8); hipMalloc(&of, 64 * 4); hipMalloc(&c, 8);
    const int iters = 1024;
    long long h;
    hipLaunchKernelGGL((chain<double, 0>), dim3(1), dim3(64), 0, 0, od, c, 1.0, 1e-9, iters);
    hipLaunchKernelGGL((chain<double, 0>), dim3(1), dim3(64), 0, 0, od, c, 1.0, 1e-9, iters);
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("{\"op\": \"f64 add (2 per step)\", \"memtime_ticks_per_add\": %.3f}\n", (double)h / (iters * 64.0 * 2));
    hipLaunchKernelGGL((chain<float, 0>), dim3(1), dim3(64), 0, 0, of, c, 1.0f, 1e-9f, iters);
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("{\"op\": \"f32 add (2 per step)\", \"memtime_ticks_per_add\": %.3f}\n", (double)h / (iters * 64.0 * 2));
    hipLaunchKernelGGL((chain<double, 1>), dim3(1), dim3(64), 0, 0, od, c, 1.0, 0.999999, iters);
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("{\"op\": \"f64 fma\", \"memtime_ticks_per_op\": %.3f}\n", (double)h / (iters * 64.0));
    // wall clock: time the f64 chain with events
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((chain<double, 0>), dim3(1), dim3(64), 0, 0, od, c, 1.0, 1e-9, iters * 16);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("{\"op\": \"f64 add wall\", \"ns_per_add\": %.3f}\n", ms * 1e6 / (iters * 16 * 64.0 * 2));
    return 0;
}
