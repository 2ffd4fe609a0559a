// pt_math.h — the bit-reproducible fp32 math contract shared by the HIP kernel
// and the host-side scene code of the MI355X path tracer.
//
// Why this exists: the reference kernel (raytrace_comp.comp) is Monte-Carlo
// path tracing.  One ULP of difference in a direction flips hit/miss and moves
// a pixel by up to intensity/spp, so "match within 1e-4 per channel" is only
// robustly reachable if the device reproduces the CPU oracle bit for bit.
// Every function here is therefore written with IEEE +,-,*,/,sqrt only, in a
// fixed evaluation order, and MUST be compiled with -ffp-contract=off and
// without fast-math (correctly rounded fp32 div/sqrt are hipcc's default on
// gfx950; the build passes -fhip-fp32-correctly-rounded-divide-sqrt anyway).
//
// GLSL built-ins have implementation-defined precision, so the reference
// leaves sin/cos/acos/log/exp/tan unspecified.  We pin them to the classic
// fdlibm-style float kernels (range reduction + minimax polynomial / rational
// approximation, ≈1 ulp on the domains the shader uses; polynomials as
// explicit fma Horner chains) — the oracle's
// oracle/glsl_math.h states the same algorithms and tests/test_math.py
// checks the two agree bitwise and stay within a few ulp of libm.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_FN __host__ __device__ static inline

namespace ptm {

PT_FN uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
PT_FN float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// GLSL min/max/abs/floor/sqrt on floats.  fmin/fmax follow IEEE minNum
// (a NaN operand yields the other operand): the AABB slab test hits 0*inf=NaN
// when the origin lies on a slab plane with a zero direction component, and
// GLSL leaves min/max undefined there.  Oracle: oracle/glsl_math.h gm_fmin.
PT_FN float fmin_(float a, float b) { return __builtin_fminf(a, b); }
PT_FN float fmax_(float a, float b) { return __builtin_fmaxf(a, b); }
PT_FN float fabs_(float a) { return __builtin_fabsf(a); }
PT_FN float sqrt_(float a) { return __builtin_sqrtf(a); }
PT_FN float floor_(float a) { return __builtin_floorf(a); }
// explicit fused multiply-add (one rounding; -ffp-contract=off never forms it)
PT_FN float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// ------------------------------------------------- fast exact quotients ----
// Device code may evaluate a quotient through the hardware reciprocal
// estimate plus fma refinement instead of the ~11-instruction IEEE division
// sequence, but only where the result is identical to the IEEE quotient:
// rcp_ is checked against 1.0f/x for all 2^32 inputs, and every unary
// function below that uses qdiv_ internally is checked against its IEEE
// definition (FAST=false) for all 2^32 inputs (tests/test_math.py,
// pt_selftest_exhaustive).  Host code (and FAST=false) divides.
#if defined(__HIP_DEVICE_COMPILE__)
#define PT_FAST_DEV 1
#else
#define PT_FAST_DEV 0
#endif

// RN(1/x): estimate y ~ 1/x (1 ulp), e = 1 - x*y exactly enough in one fma,
// y + e*y rounds to 1/x.  Zeros, infinities, NaNs, subnormal x and |x| so
// large that 1/x is subnormal take the IEEE division.
PT_FN float rcp_(float x) {
#if PT_FAST_DEV
  const float ax = __builtin_fabsf(x);
  if (ax >= 0x1p-126f && ax <= 0x1p126f) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
  }
#endif
  return 1.0f / x;
}

// a/b via q = a*RN(1/b) and one remainder correction (Markstein); used only
// inside functions verified exhaustively against their IEEE definitions.
PT_FN float qdiv_(float a, float b) {
#if PT_FAST_DEV
  const float y = rcp_(b);
  const float q = a * y;
  const float r = __builtin_fmaf(-b, q, a);
  return __builtin_fmaf(r, y, q);
#else
  return a / b;
#endif
}
#define PT_DIV(FAST, a, b) ((FAST) ? qdiv_((a), (b)) : (a) / (b))

// ---------------------------------------------------------------- logf ----
// fdlibm e_logf.c algorithm: x = 2^k (1+f), f in [sqrt(2)/2-1, sqrt(2)-1),
// log(1+f) = f - (hfsq - s*(hfsq+R)), s = f/(2+f).  Subnormals (1e-38 is one:
// raytrace_comp.comp:220) are pre-scaled by 2^25.
template <bool FAST>
PT_FN float log_impl(float x) {
  uint32_t ix = f2u(x);
  int k = 0;
  if (ix < 0x00800000u) {               // +0 or +subnormal
    if (ix == 0u) return -__builtin_inff();
    x = x * 0x1.0p25f;
    ix = f2u(x);
    k = -25;
  }
  if (ix >= 0x7f800000u) {              // +inf, NaN or negative
    if (ix == 0x7f800000u) return x;
    return __builtin_nanf("");
  }
  k += (int)(ix >> 23) - 127;
  ix &= 0x007fffffu;
  uint32_t i = (ix + 0x4afb20u) & 0x00800000u;  // mantissa >= sqrt(2) ?
  x = u2f(ix | (i ^ 0x3f800000u));
  k += (int)(i >> 23);
  const float f = x - 1.0f;
  const float s = PT_DIV(FAST, f, 2.0f + f);
  const float dk = (float)k;
  const float z = s * s;
  const float w = z * z;
  const float t1 = w * fma_(w, fma_(w, 0x1.39a09ep-3f, 0x1.c71c52p-3f), 0x1.99999ap-2f);
  const float t2 = z * fma_(w, fma_(w, fma_(w, 0x1.2f112ep-3f, 0x1.74664ap-3f), 0x1.24924ap-2f), 0x1.555556p-1f);
  const float R = t2 + t1;
  const float hfsq = 0.5f * f * f;
  return fma_(dk, 0x1.62e3p-1f, -((hfsq - fma_(s, hfsq + R, dk * 0x1.2fefa2p-17f)) - f));
}
PT_FN float log_(float x) { return log_impl<PT_FAST_DEV>(x); }

// ---------------------------------------------------------------- expf ----
// fdlibm e_expf.c algorithm: k = round(x/ln2), r = hi - lo, rational kernel,
// then scale by 2^k (two steps below the normal range).
template <bool FAST>
PT_FN float exp_impl(float x) {
  if (x != x) return x;
  if (x > 88.72283935546875f) return __builtin_inff();
  if (x < -103.972084045410156f) return 0.0f;
  const float kf = floor_(x * 0x1.715476p+0f + 0.5f);
  const int k = (int)kf;
  const float hi = fma_(-kf, 0x1.62e4p-1f, x);
  const float lo = kf * 0x1.7f7d1cp-20f;
  const float r = hi - lo;
  const float t = r * r;
  const float c = fma_(-t, fma_(t, fma_(t, fma_(t, fma_(t, 0x1.637698p-25f, -0x1.bbd41cp-20f), 0x1.1566aap-14f),
                                      -0x1.6c16c2p-9f), 0x1.555556p-3f), r);
  const float y = 1.0f - ((lo - PT_DIV(FAST, r * c, 2.0f - c)) - hi);
  if (k >= -125) {
    if (k > 127) return y * u2f((uint32_t)(127 + 127) << 23) * u2f((uint32_t)(k - 127 + 127) << 23);
    return y * u2f((uint32_t)(k + 127) << 23);
  }
  return (y * u2f((uint32_t)(k + 100 + 127) << 23)) * 0x1.0p-100f;
}
PT_FN float exp_(float x) { return exp_impl<PT_FAST_DEV>(x); }

// ------------------------------------------------------- sin/cos kernels ----
// fdlibm k_sin/k_cos polynomials on |r| <= pi/4.
PT_FN float ksin_(float x) {
  const float z = x * x;
  const float v = z * x;
  const float r = fma_(z, fma_(z, fma_(z, fma_(z, 0x1.5d93a6p-33f, -0x1.ae5e68p-26f), 0x1.71de36p-19f),
                               -0x1.a01a02p-13f), 0x1.111112p-7f);
  return fma_(v, fma_(z, r, -0x1.555556p-3f), x);
}
PT_FN float kcos_(float x) {
  const float z = x * x;
  const float r = z * fma_(z, fma_(z, fma_(z, fma_(z, fma_(z, -0x1.8fae9cp-37f, 0x1.1ee9ecp-29f), -0x1.27e4f8p-22f),
                                          0x1.a01a02p-16f), -0x1.6c16c2p-10f), 0x1.555556p-5f);
  const float hz = 0.5f * z;
  const float w = 1.0f - hz;
  return w + fma_(z, r, (1.0f - w) - hz);
}
// Cody–Waite reduction by pi/2 in three parts (12+12+24 bits): exact products
// for |quadrant| < 4096, i.e. |x| < ~6400 — the shader only feeds [0, 2*pi].
PT_FN float reduce_(float x, int* q) {
  const float jf = floor_(x * 0x1.45f306p-1f + 0.5f);
  *q = (int)jf;
  return fma_(-jf, 0x1.4442d2p-24f, fma_(-jf, 0x1.fb4p-12f, fma_(-jf, 0x1.92p+0f, x)));
}
PT_FN float sin_(float x) {
  int q;
  const float r = reduce_(x, &q);
  switch (q & 3) {
    case 0: return ksin_(r);
    case 1: return kcos_(r);
    case 2: return -ksin_(r);
    default: return -kcos_(r);
  }
}
PT_FN float cos_(float x) {
  int q;
  const float r = reduce_(x, &q);
  switch (q & 3) {
    case 0: return kcos_(r);
    case 1: return -ksin_(r);
    case 2: return -kcos_(r);
    default: return ksin_(r);
  }
}
// sin and cos of one argument sharing the reduction: bitwise the same as
// sin_(x) and cos_(x).
PT_FN void sincos_(float x, float* s, float* c) {
  int q;
  const float r = reduce_(x, &q);
  const float ks = ksin_(r), kc = kcos_(r);
  switch (q & 3) {
    case 0: *s = ks; *c = kc; break;
    case 1: *s = kc; *c = -ks; break;
    case 2: *s = -ks; *c = -kc; break;
    default: *s = -kc; *c = ks; break;
  }
}
PT_FN float tan_(float x) { return sin_(x) / cos_(x); }

// ---------------------------------------------------------------- acosf ----
// fdlibm e_acosf.c algorithm (rational approximation of asin, three ranges).
template <bool FAST>
PT_FN float acos_rat_(float z) {
  const float p = z * fma_(z, fma_(z, fma_(z, fma_(z, fma_(z, 0x1.23de1p-15f, 0x1.9efe08p-11f), -0x1.48228cp-5f),
                                          0x1.9c155p-3f), -0x1.4d612p-2f), 0x1.555556p-3f);
  const float q = fma_(z, fma_(z, fma_(z, fma_(z, 0x1.3b8c5cp-4f, -0x1.6066c2p-1f), 0x1.02ae5ap+1f), -0x1.33a272p+1f), 1.0f);
  return PT_DIV(FAST, p, q);
}
template <bool FAST>
PT_FN float acos_impl(float x) {
  const float pio2_hi = 0x1.921fb4p+0f, pio2_lo = 0x1.4442d0p-24f, pi_ = 0x1.921fb4p+1f;
  const uint32_t ix = f2u(x) & 0x7fffffffu;
  if (ix == 0x3f800000u) return (f2u(x) >> 31) ? pi_ + 2.0f * pio2_lo : 0.0f;
  if (ix > 0x3f800000u) return __builtin_nanf("");
  if (ix < 0x3f000000u) {                      // |x| < 0.5
    if (ix <= 0x32800000u) return pio2_hi + pio2_lo;
    const float z = x * x;
    const float r = acos_rat_<FAST>(z);
    return pio2_hi - (x - fma_(-x, r, pio2_lo));
  }
  if (f2u(x) >> 31) {                          // x <= -0.5
    const float z = (1.0f + x) * 0.5f;
    const float s = sqrt_(z);
    const float r = acos_rat_<FAST>(z);
    const float w = fma_(r, s, -pio2_lo);
    return pi_ - 2.0f * (s + w);
  }
  const float z = (1.0f - x) * 0.5f;           // x >= 0.5
  const float s = sqrt_(z);
  const float df = u2f(f2u(s) & 0xfffff000u);
  const float c = PT_DIV(FAST, fma_(-df, df, z), s + df);
  const float r = acos_rat_<FAST>(z);
  const float w = fma_(r, s, c);
  return 2.0f * (df + w);
}
PT_FN float acos_(float x) { return acos_impl<PT_FAST_DEV>(x); }

// -------------------------------------------------------------- vec3 ops ----
struct v3 { float x, y, z; };
PT_FN v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_FN v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_FN v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_FN v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_FN v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
PT_FN v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
// GLSL dot/cross/length/normalize, evaluated left to right, no contraction.
PT_FN float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_FN v3 cross(v3 a, v3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
PT_FN float length(v3 a) { return sqrt_(dot(a, a)); }
PT_FN v3 normalize(v3 a) { return muls(a, rcp_(sqrt_(dot(a, a)))); }

// GLSL radians(): deg * float(pi/180).
PT_FN float radians_(float deg) { return deg * 0x1.1df46ap-6f; }

// ----------------------------------------------------------------- RNG ------
// raytrace_comp.comp:209-216 (PCG-style LCG + RXS-M-XS output).  The divisor
// literal 4294967295.0 is a GLSL *float* literal, i.e. 2^32 exactly.
// The state update of rng_next alone: n draws whose values are never used
// (a direction the shader samples and never traces) still advance the stream.
PT_FN void rng_skip(uint32_t* s, int n) {
  for (int i = 0; i < n; ++i) *s = *s * 747796405u + 2891336453u;
}
PT_FN float rng_next(uint32_t* s) {
  *s = *s * 747796405u + 2891336453u;
  uint32_t result = ((*s >> ((*s >> 28u) + 4u)) ^ *s) * 277803737u;
  result = (result >> 22u) ^ result;
  return (float)result / 0x1.0p32f;
}

}  // namespace ptm
