// diagnostic: cycles per forward stage of the MFMA forward chain (one wave), adding the stage's pieces
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) double ldsd;
__device__ __forceinline__ long long stamp_after(double v) {
  long long t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(v)); return t;
}
__device__ __forceinline__ void pin(double& v) { asm volatile("; pin %0" : "+v"(v)); }
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
__device__ __forceinline__ double mfma4(double a, double b, double c) { return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0); }
template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int V> using IC = std::integral_constant<int, V>;
template <typename Fn, int... S> __device__ __forceinline__ void each(Fn&& fn, std::integer_sequence<int, S...>) { (fn(IC<S>{}), ...); }
constexpr int DF = 8, NST = 64;
template <int MODE>
__device__ long long run(const double* F, ldsd* lds, int lane) {
  const int g = lane >> 4, c = lane & 15, cb = (c >> 2) & 3;
  const bool fst = c == 0, cb0 = cb == 0, cb1 = cb == 1;
  double xb0 = 0.1 * lane, xb1 = 0.2, xb2 = g == 3 ? 1.0 : 0.0;
  const d4 z4 = {0, 0, 0, 0};
  double fr[DF][4];
  auto fissue = [&](double* rs, int k) {
    const double* fb = F + (size_t)(k & 63) * 256 + lane;
    rs[0] = fb[0]; rs[1] = fb[64]; rs[2] = fb[128]; rs[3] = F[(size_t)(k & 63) * 256 + 192 + (lane & 31)];
  };
  for (int j = 0; j < DF; ++j) fissue(fr[j], j);
  const double m0c = F[lane], m1c = F[64 + lane], m2c = F[128 + lane], cqc = F[192 + lane];
  long long t0 = stamp_after(xb0 + m0c + fr[DF - 1][3]);
  for (int q0 = 0; q0 < NST; q0 += DF) {
    each([&](auto Jc) {
      constexpr int J = decltype(Jc)::value;
      double m0 = m0c, m1 = m1c, m2 = m2c, cq = cqc;
      if constexpr (MODE >= 3) { m0 = fr[J][0]; m1 = fr[J][1]; m2 = fr[J][2]; cq = fr[J][3]; fissue(fr[J], q0 + J + DF); }
      d4 D = mfma(m0, xb0, z4); D = mfma(m1, xb1, D); D = mfma(m2, xb2, D);
      double P = 0.0;
      if constexpr (MODE >= 1) {
        const double xbc = cb0 ? xb0 : cb1 ? xb1 : xb2;
        P = mfma4(cq, xbc, 0.0);
        P += dpp64<0x124>(P); P += dpp64<0x128>(P);
      }
      xb0 = D[0] * 1e-3; xb1 = D[1] * 1e-3; xb2 = D[2];
      if constexpr (MODE >= 2) {
        ldsd* xo = lds + ((q0 + J) & 31) * 16;
        *(fst ? xo + g : lds + 600) = D[0];
        *(fst ? xo + 4 + g : lds + 600) = D[1];
        *(fst ? xo + 8 + g : lds + 600) = D[2];
        *(fst ? xo + 12 + g : lds + 600) = D[3];
        *(fst ? xo + 520 + g : lds + 600) = P;
      } else {
        xb2 += P * 1e-30;
      }
    }, std::make_integer_sequence<int, DF>{});
  }
  long long t1 = stamp_after(xb0 + xb1 + xb2);
  lds[lane] = xb0 + xb1 + xb2;
  return t1 - t0;
}
__global__ void probe(long long* cyc, const double* F) {
  __shared__ double lds_[640];
  ldsd* lds = (ldsd*)lds_;
  const int lane = threadIdx.x;
  long long r0 = run<0>(F, lds, lane), r1 = run<1>(F, lds, lane), r2 = run<2>(F, lds, lane), r3 = run<3>(F, lds, lane);
  if (lane == 0) { cyc[0] = r0; cyc[1] = r1; cyc[2] = r2; cyc[3] = r3; }
}
int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1;
  double* F; long long* c; hipMalloc(&c, 8 * 4 * 2048); hipMalloc(&F, 8 * 256 * 64 * 2048);
  hipMemset(F, 0, 8 * 256 * 64 * 2048);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, c, F);
  hipDeviceSynchronize();
  long long h[4]; hipMemcpy(h, c, 32, hipMemcpyDeviceToHost);
  const char* n[4] = {"chain", "+ C x (mfma4, dpp)", "+ 5 LDS stores", "+ streamed operands (DF 8)"};
  for (int i = 0; i < 4; ++i) printf("blocks %d  %-26s %.1f cycles / stage\n", blocks, n[i], h[i] / (double)NST);
  return 0;
}
