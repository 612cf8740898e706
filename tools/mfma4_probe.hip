// diagnostic: operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 on gfx950, and its dependent latency
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(double* out, long long* cyc) {
  const int lane = threadIdx.x;
  for (int L = 0; L < 64; ++L) {
    const double a = lane == L ? 1.0 : 0.0, b = lane + 1.0;
    out[L * 64 + lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  }
  for (int L = 0; L < 64; ++L) {  // B one-hot, A distinct
    const double b = lane == L ? 1.0 : 0.0, a = lane + 1.0;
    out[4096 + L * 64 + lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  }
  // dependent chains: 16 x 4x4x4 and 16 x 16x16x4
  double x = lane * 1e-3;
  long long t0 = clock64();
  for (int i = 0; i < 16; ++i) x = __builtin_amdgcn_mfma_f64_4x4x4f64(x, 1.0001, x, 0, 0, 0);
  long long t1 = clock64();
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 y = {x, x, x, x};
  for (int i = 0; i < 16; ++i) y = __builtin_amdgcn_mfma_f64_16x16x4f64(y[0], 1.0001, y, 0, 0, 0);
  long long t2 = clock64();
  d4 z0 = y, z1 = y;
  for (int i = 0; i < 16; ++i) { z0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, 1.0001, z0, 0, 0, 0); z1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, 1.0002, z1, 0, 0, 0); }
  long long t3 = clock64();
  double w0 = x, w1 = x, w2 = x, w3 = x;
  for (int i = 0; i < 16; ++i) { w0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, 1.0001, w0, 0, 0, 0); w1 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, 1.0002, w1, 0, 0, 0); w2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, 1.0003, w2, 0, 0, 0); w3 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, 1.0004, w3, 0, 0, 0); }
  long long t4 = clock64();
  out[8192 + lane] = y[1] + z0[2] + z1[3] + w0 + w1 + w2 + w3;
  if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; }
}
int main() {
  double* d; long long* c; hipMalloc(&d, 8 * 8256); hipMalloc(&c, 64);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, c);
  static double h[8256]; long long hc[4];
  hipMemcpy(h, d, 8 * 8256, hipMemcpyDeviceToHost); hipMemcpy(hc, c, 32, hipMemcpyDeviceToHost);
  printf("cycles: 16 dep 4x4x4 %lld | 16 dep 16x16x4 %lld | 2x16 indep 16x16x4 %lld | 4x16 indep 4x4x4 %lld\n", hc[0], hc[1], hc[2], hc[3]);
  for (int t = 0; t < 2; ++t)
    for (int L = 0; L < 64; ++L) {
      printf("%c%02d:", t ? 'B' : 'A', L);
      for (int m = 0; m < 64; ++m) printf(" %g", h[t * 4096 + L * 64 + m]);
      printf("\n");
    }
  return 0;
}
