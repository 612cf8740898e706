// Diagnostic: effective shader clock under sustained f32 / f64 MFMA load on 1..all CUs (clock64 cycles
// per s_memrealtime tick, the 100 MHz constant clock), to tell power-capped clocks from kernel stalls.
// build: hipcc --offload-arch=gfx950 -O2 tools/clock_probe.hip -o tools/_clock_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef double d4v __attribute__((ext_vector_type(4)));

template <int F64>
__global__ __launch_bounds__(256) void burn(double* out, int iters) {
    const long long c0 = clock64(), t0 = __builtin_amdgcn_s_memrealtime();
    f16v a = {};
    d4v b = {};
    float x = threadIdx.x * 1e-3f;
    double y = threadIdx.x * 1e-3;
    for (int i = 0; i < iters; ++i) {
        if (F64) {
            b = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, b, 0, 0, 0);
            b = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, b, 0, 0, 0);
        } else {
            a = __builtin_amdgcn_mfma_f32_32x32x2f32(x, x, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_32x32x2f32(x, x, a, 0, 0, 0);
        }
    }
    const long long c1 = clock64(), t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x * 4 + 0] = (double)(c1 - c0);
        out[blockIdx.x * 4 + 1] = (double)(t1 - t0);
        out[blockIdx.x * 4 + 2] = F64 ? b[0] : a[0];
    }
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    double* d;
    (void)hipMalloc(&d, 8 * 4 * 4096);
    std::vector<double> h(4 * 4096);
    printf("{\"cus\": %d", ncu);
    for (int f64 = 0; f64 < 2; ++f64)
        for (int nb : {ncu / 8, ncu / 2, ncu, 2 * ncu}) {
            const int iters = 20000;
            for (int rep = 0; rep < 2; ++rep) {
                if (f64) hipLaunchKernelGGL(burn<1>, nb, 256, 0, 0, d, iters);
                else hipLaunchKernelGGL(burn<0>, nb, 256, 0, 0, d, iters);
                (void)hipDeviceSynchronize();
            }
            (void)hipMemcpy(h.data(), d, 8 * 4 * nb, hipMemcpyDeviceToHost);
            double cyc = 0, tick = 0;
            for (int b = 0; b < nb; ++b) { cyc += h[b * 4]; tick += h[b * 4 + 1]; }
            printf(", \"%s_wg%d_mhz\": %.0f", f64 ? "f64" : "f32", nb, cyc / tick * 100.0);
        }
    printf("}\n");
    return 0;
}
