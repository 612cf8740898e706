// diagnostic: issue interval / dependent latency of the f64 MFMAs on gfx950 (one wave)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ long long stamp_after(double v) {
  long long t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(v)); return t;
}
__device__ __forceinline__ void pin(double& v) { asm volatile("; pin %0" : "+v"(v)); }
template <int R>
__device__ __forceinline__ void pin4(d4& v) { double a = v[0], b = v[1], c = v[2], d = v[3]; asm volatile("; pin %0 %1 %2 %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)); v = d4{a, b, c, d}; }
__global__ void lat(double* out, long long* cyc) {
  const int lane = threadIdx.x;
  double x = lane * 1e-3;
  long long t[8];
  t[0] = stamp_after(x); pin(x);
  for (int i = 0; i < 32; ++i) x = __builtin_amdgcn_mfma_f64_4x4x4f64(x, 1.0001, x, 0, 0, 0);   // dependent via C and A
  t[1] = stamp_after(x); pin(x);
  for (int i = 0; i < 32; ++i) x = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, 1.0001, x, 0, 0, 0);  // dependent via C only
  t[2] = stamp_after(x); pin(x);
  double w0 = x, w1 = x + 1, w2 = x + 2, w3 = x + 3;
  for (int i = 0; i < 32; ++i) { w0 = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, 1.0001, w0, 0, 0, 0); w1 = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, 1.0002, w1, 0, 0, 0); w2 = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, 1.0003, w2, 0, 0, 0); w3 = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, 1.0004, w3, 0, 0, 0); }
  x = w0 + w1 + w2 + w3;
  t[3] = stamp_after(x); pin(x);
  d4 y = {x, x, x, x};
  for (int i = 0; i < 32; ++i) y = __builtin_amdgcn_mfma_f64_16x16x4f64(1.0, 1.0001, y, 0, 0, 0);   // dependent via C
  t[4] = stamp_after(y[0] + y[3]); x = y[1]; pin(x);
  d4 z0 = {x, x, x, x}, z1 = z0;
  for (int i = 0; i < 32; ++i) { z0 = __builtin_amdgcn_mfma_f64_16x16x4f64(1.0, 1.0001, z0, 0, 0, 0); z1 = __builtin_amdgcn_mfma_f64_16x16x4f64(1.0, 1.0002, z1, 0, 0, 0); }
  t[5] = stamp_after(z0[0] + z1[3]); x = z0[2]; pin(x);
  for (int i = 0; i < 32; ++i) { d4 q = {0, 0, 0, 0}; q = __builtin_amdgcn_mfma_f64_16x16x4f64(x, 1.0001, q, 0, 0, 0); x = q[0]; }  // result -> A operand
  t[6] = stamp_after(x); pin(x);
  for (int i = 0; i < 32; ++i) x = fma(x, 1.0001, 1e-9);  // VALU f64 dependent
  t[7] = stamp_after(x);
  out[lane] = x;
  if (lane == 0) for (int i = 0; i < 7; ++i) cyc[i] = t[i + 1] - t[i];
}
int main() {
  double* d; long long* c; hipMalloc(&d, 8 * 64); hipMalloc(&c, 64);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, d, c);
  long long h[7]; hipMemcpy(h, c, 56, hipMemcpyDeviceToHost);
  const char* n[7] = {"4x4x4 dep(A,C)", "4x4x4 dep C", "4x4x4 4 indep", "16x16x4 dep C", "16x16x4 2 indep", "16x16x4 D->A", "v_fma_f64 dep"};
  for (int i = 0; i < 7; ++i) printf("%-18s %6lld cycles / 32 = %.1f\n", n[i], h[i], h[i] / 32.0);
  return 0;
}
