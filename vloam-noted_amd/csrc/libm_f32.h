// libm_f32.h — glibc's single-precision atanf / atan2f, restated for the device.
//
// The reference computes every point's azimuth with the float overload of atan2
// (scan_registration.h:58 `using std::atan2`; scan_registration.cpp:185,187,263) and its
// elevation with atan(float) (:217).  On the reference's x86-64 Linux hosts those resolve to
// glibc's generic flt-32 implementations (sysdeps/ieee754/flt-32/s_atanf.c and e_atan2f.c, the
// fdlibm algorithms; unchanged from glibc 2.27 through 2.39, no x86-64 multiarch variant).
// The device's own atan2f (ocml) differs from them by up to an ulp, which moves `intensity`
// (= scanID + 0.1 * relTime) off the reference's bits and, at the 0.5 boundaries of the ring
// rule (:243-246) or at the halfPassed knife edge (:276,:288), moves a point to another ring
// or by a whole revolution in relTime.  These restatements use only IEEE single-precision
// + - * / (correctly rounded on gfx950, compiled with -ffp-contract=off) and integer tests on
// the bit patterns, so they return glibc's bits.  tests/test_host_models.py (tests/cxx/libm_f32_check.cpp) checks them against
// the host's glibc on ~10^7 inputs, the special values included.
//
// Constants are the decimal literals of the glibc sources, converted double -> float exactly
// as the C compiler does there (the hex words in glibc's comments are not always the values).
#pragma once
#include <stdint.h>

namespace loam {

__host__ __device__ inline int32_t f32_word(float x) { return __builtin_bit_cast(int32_t, x); }
__host__ __device__ inline float f32_from(int32_t w) { return __builtin_bit_cast(float, w); }
__host__ __device__ inline float f32_abs(float x) { return f32_from(f32_word(x) & 0x7fffffff); }

// glibc sysdeps/ieee754/flt-32/s_atanf.c (__atanf)
__host__ __device__ inline float glibc_atanf(float x) {
  const float atanhi[4] = {(float)4.6364760399e-01, (float)7.8539812565e-01, (float)9.8279368877e-01,
                           (float)1.5707962513e+00};
  const float atanlo[4] = {(float)5.0121582440e-09, (float)3.7748947079e-08, (float)3.4473217170e-08,
                           (float)7.5497894159e-08};
  const float aT0 = (float)3.3333334327e-01, aT1 = (float)-2.0000000298e-01, aT2 = (float)1.4285714924e-01,
              aT3 = (float)-1.1111110449e-01, aT4 = (float)9.0908870101e-02, aT5 = (float)-7.6918758452e-02,
              aT6 = (float)6.6610731184e-02, aT7 = (float)-5.8335702866e-02, aT8 = (float)4.9768779427e-02,
              aT9 = (float)-3.6531571299e-02, aT10 = (float)1.6285819933e-02;
  const float one = 1.0f;
  const int32_t hx = f32_word(x);
  const int32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;  // NaN
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3ee00000) {  // |x| < 0.4375
    if (ix < 0x31000000) return x;  // |x| < 2^-29
    id = -1;
  } else {
    x = f32_abs(x);
    if (ix < 0x3f980000) {    // |x| < 1.1875
      if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
        id = 0;
        x = ((float)2.0 * x - one) / ((float)2.0 + x);
      } else {  // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - one) / (x + one);
      }
    } else {
      if (ix < 0x401c0000) {  // |x| < 2.4375
        id = 2;
        x = (x - (float)1.5) / (one + (float)1.5 * x);
      } else {  // 2.4375 <= |x| < 2^25
        id = 3;
        x = -(float)1.0 / x;
      }
    }
  }
  float z = x * x;
  const float w = z * z;
  const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -z : z;
}

// glibc sysdeps/ieee754/flt-32/e_atan2f.c (__ieee754_atan2f)
__host__ __device__ inline float glibc_atan2f(float y, float x) {
  const float tiny = (float)1.0e-30, zero = 0.0f, pi_o_4 = (float)7.8539818525e-01,
              pi_o_2 = (float)1.5707963705e+00, pi = (float)3.1415927410e+00, pi_lo = (float)-8.7422776573e-08;
  const int32_t hx = f32_word(x), ix = hx & 0x7fffffff;
  const int32_t hy = f32_word(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;  // NaN
  if (hx == 0x3f800000) return glibc_atanf(y);           // x = 1.0
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);     // 2 * sign(x) + sign(y)
  if (iy == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return (float)3.0 * pi_o_4 + tiny;
        default: return (float)-3.0 * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0: return zero;
      case 1: return -zero;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int32_t k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + (float)0.5 * pi_lo;  // |y/x| > 2^60
  else if (hx < 0 && k < -60) z = 0.0f;         // |y|/x < -2^60
  else z = glibc_atanf(f32_abs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return f32_from(f32_word(z) ^ (int32_t)0x80000000);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

}  // namespace loam
