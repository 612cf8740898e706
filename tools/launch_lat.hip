// Diagnostic: host-side latency floors of the C2 call path on this box -- empty-kernel launch + sync,
// small pinned copies, copy + kernel + copy, the same captured in a hipGraph, and a 23 us spin kernel.
// build: hipcc --offload-arch=gfx950 -O2 tools/launch_lat.hip -o tools/_launch_lat
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void empty_k(float* p) {
    if (threadIdx.x == 0 && p) p[0] += 1.0f;
}
__global__ void spin_k(float* p, long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) p[0] += 1.0f;
}

template <class F>
static double med_us(F f, int n = 400) {
    std::vector<double> t(n);
    for (int i = 0; i < 20; ++i) f();
    for (int i = 0; i < n; ++i) {
        auto a = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[n / 2];
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    float *d, *h;
    (void)hipMalloc(&d, 4096);
    (void)hipHostMalloc(&h, 4096, hipHostMallocDefault);
    const size_t n = 132 * 4;
    printf("{\"launch_sync_us\": %.2f", med_us([&] { hipLaunchKernelGGL(empty_k, 1, 64, 0, s, d); (void)hipStreamSynchronize(s); }));
    printf(", \"h2d_sync_us\": %.2f", med_us([&] { (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s); (void)hipStreamSynchronize(s); }));
    printf(", \"h2d_k_d2h_sync_us\": %.2f", med_us([&] {
        (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s);
        hipLaunchKernelGGL(empty_k, 1, 64, 0, s, d);
        (void)hipMemcpyAsync(h + 512, d, n, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }));
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(empty_k, 1, 64, 0, s, d);
    (void)hipMemcpyAsync(h + 512, d, n, hipMemcpyDeviceToHost, s);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    printf(", \"graph_sync_us\": %.2f", med_us([&] { (void)hipGraphLaunch(ge, s); (void)hipStreamSynchronize(s); }));
    const long long cyc = 23LL * 100;  // clock64 at 100 MHz: 23 us
    printf(", \"spin23_launch_sync_us\": %.2f", med_us([&] { hipLaunchKernelGGL(spin_k, 1, 64, 0, s, d, cyc); (void)hipStreamSynchronize(s); }));
    printf(", \"spin23_h2d_k_d2h_us\": %.2f}\n", med_us([&] {
        (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s);
        hipLaunchKernelGGL(spin_k, 1, 64, 0, s, d, cyc);
        (void)hipMemcpyAsync(h + 512, d, n, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }));
    return 0;
}
