// Range-reduced fp32 sine/cosine for the SIREN activations (sin(w0 * a), w0 = 20) and the positional
// embedding (sin(2^f * proj), |arg| up to tens of radians), reference activation.py:12-13 and
// embeddings.py:106-111.
//
// CDNA's v_sin_f32 / v_cos_f32 (and __sinf) take a revolution argument and are inaccurate beyond a
// few periods, so they cannot meet the 1e-5 parity bar.  This is a 3-constant Cody-Waite reduction
// by pi/2 with fused multiply-adds, then minimax polynomials on [-pi/4, pi/4]: ~1 ulp for
// |x| < 2^17, one shared reduction for sin and cos.  Larger |x| (never reached by a sane network)
// take the libm/ocml path, so the function is correct everywhere.
#pragma once

#if defined(__HIPCC__)
#define SDFN_HD __host__ __device__ __forceinline__
#else
#define SDFN_HD static inline
#include <math.h>
#endif

SDFN_HD void sdfn_sincosf(float x, float* s_out, float* c_out) {
#ifndef SDF_FAST_SIN_ONLY  // diagnostic build: no large-argument path (wrong beyond |x| = 2^17)
    if (!(fabsf(x) < 131072.0f)) {  // also NaN / inf
#if defined(__HIP_DEVICE_COMPILE__)
        sincosf(x, s_out, c_out);
#else
        *s_out = sinf(x);
        *c_out = cosf(x);
#endif
        return;
    }
#endif
    const float q = rintf(x * 0.636619772367581343f);  // x * 2/pi
    // pi/2 = C1 + C2 + C3, C1/C2 exact fp32
    float r = fmaf(q, -1.57079637050628662109375f, x);
    r = fmaf(q, 4.37113882867379289e-8f, r);
    r = fmaf(q, 1.71512451e-15f, r);  // C2 = -4.3711388e-8, C3 = -1.7151245e-15
    const float r2 = r * r;
    // sin on [-pi/4, pi/4]
    float ps = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = fmaf(r2, ps, -1.6666654611e-1f);
    const float sr = fmaf(r * r2, ps, r);
    // cos on [-pi/4, pi/4]
    float pc = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = fmaf(r2, pc, 4.166664568298827e-2f);
    const float cr = fmaf(r2 * r2, pc, fmaf(r2, -0.5f, 1.0f));
    const int qi = (int)q;
    const float s1 = (qi & 1) ? cr : sr;
    const float c1 = (qi & 1) ? sr : cr;
    *s_out = (qi & 2) ? -s1 : s1;
    *c_out = ((qi + 1) & 2) ? -c1 : c1;
}

#if defined(__HIPCC__)
// Two arguments at once on the packed fp32 pipe (v_pk_fma_f32 / v_pk_mul_f32): the same operations as
// sdfn_sincosf element by element (IEEE fma and products per element), so the same bits.
typedef float sdfn_f2 __attribute__((ext_vector_type(2)));
// the large-argument path out of line (it is never taken by a sane network; inlined at every pair it
// doubled the epilogues' code)
static __device__ __attribute__((noinline)) float4 sdfn_sincosf2_slow(float x0, float x1) {
    float4 r;
    sdfn_sincosf(x0, &r.x, &r.y);
    sdfn_sincosf(x1, &r.z, &r.w);
    return r;
}
__device__ __forceinline__ void sdfn_sincosf2(float x0, float x1, float* s0, float* c0, float* s1, float* c1) {
#ifndef SDF_FAST_SIN_ONLY
    if (!(fabsf(x0) < 131072.0f) || !(fabsf(x1) < 131072.0f)) {
        const float4 r = sdfn_sincosf2_slow(x0, x1);
        *s0 = r.x;
        *c0 = r.y;
        *s1 = r.z;
        *c1 = r.w;
        return;
    }
#endif
    const sdfn_f2 x = {x0, x1};
    const sdfn_f2 t = x * 0.636619772367581343f;
    const sdfn_f2 q = {rintf(t.x), rintf(t.y)};
    sdfn_f2 r = __builtin_elementwise_fma(q, (sdfn_f2)(-1.57079637050628662109375f), x);
    r = __builtin_elementwise_fma(q, (sdfn_f2)(4.37113882867379289e-8f), r);
    r = __builtin_elementwise_fma(q, (sdfn_f2)(1.71512451e-15f), r);
    const sdfn_f2 r2 = r * r;
    sdfn_f2 ps = __builtin_elementwise_fma(r2, (sdfn_f2)(-1.9515295891e-4f), (sdfn_f2)(8.3321608736e-3f));
    ps = __builtin_elementwise_fma(r2, ps, (sdfn_f2)(-1.6666654611e-1f));
    const sdfn_f2 sr = __builtin_elementwise_fma(r * r2, ps, r);
    sdfn_f2 pc = __builtin_elementwise_fma(r2, (sdfn_f2)(2.443315711809948e-5f), (sdfn_f2)(-1.388731625493765e-3f));
    pc = __builtin_elementwise_fma(r2, pc, (sdfn_f2)(4.166664568298827e-2f));
    const sdfn_f2 cr = __builtin_elementwise_fma(r2 * r2, pc, __builtin_elementwise_fma(r2, (sdfn_f2)(-0.5f), (sdfn_f2)(1.0f)));
    const int q0 = (int)q.x, q1 = (int)q.y;
    const float sa = (q0 & 1) ? cr.x : sr.x, ca = (q0 & 1) ? sr.x : cr.x;
    const float sb = (q1 & 1) ? cr.y : sr.y, cb = (q1 & 1) ? sr.y : cr.y;
    *s0 = (q0 & 2) ? -sa : sa;
    *c0 = ((q0 + 1) & 2) ? -ca : ca;
    *s1 = (q1 & 2) ? -sb : sb;
    *c1 = ((q1 + 1) & 2) ? -cb : cb;
}
#endif
