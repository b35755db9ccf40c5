/* tools/trig_outcomes.h — the float32 quantities the action step derives from
 * sin/cos(angle) and sin/cos(angle + pi/2) (csrc/flock_step_w64.hip, actions block):
 * the forces f32((c0*k0 + c1*k1)*cc*F), f32((s0*k0 + s1*k1)*cc*F) for k0,k1 in {-1,0,1},
 * cc in {1, 1/sqrt(2)}, F in {20, 16} (Flock; TDM with the move penalty), and the melee
 * ray offsets f32(2*c0), f32(2*s0). Shared by tools/trig_check.c (host) and
 * tools/trig_gpu_check.hip (device); compile both with -ffp-contract=off. */
#pragma once
#include <stdint.h>
#include <string.h>
#ifdef __HIPCC__
#define TRIG_FN __host__ __device__ static inline
#else
#define TRIG_FN static inline
#endif

TRIG_FN uint32_t f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

TRIG_FN int f32_outcomes_differ(double c0a, double s0a, double c1a, double s1a,
                                double c0b, double s0b, double c1b, double s1b) {
  const double ccs[2] = {1.0, 0.70710678118654746 /* 1.0 / sqrt(2.0) */}, Fs[2] = {20.0, 16.0};
  int bad = 0;
  for (int k0 = -1; k0 <= 1; ++k0)
    for (int k1 = -1; k1 <= 1; ++k1)
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) {
          const double a = k0, b = k1;
          float fxa = (float)((c0a * a + c1a * b) * ccs[i] * Fs[j]);
          float fxb = (float)((c0b * a + c1b * b) * ccs[i] * Fs[j]);
          float fya = (float)((s0a * a + s1a * b) * ccs[i] * Fs[j]);
          float fyb = (float)((s0b * a + s1b * b) * ccs[i] * Fs[j]);
          fxa = 0.0f + fxa; fxb = 0.0f + fxb; fya = 0.0f + fya; fyb = 0.0f + fyb;
          bad |= f32_bits(fxa) != f32_bits(fxb) || f32_bits(fya) != f32_bits(fyb);
        }
  const float ra = (float)(2.0 * c0a), rb = (float)(2.0 * c0b);
  const float qa = (float)(2.0 * s0a), qb = (float)(2.0 * s0b);
  bad |= f32_bits(ra) != f32_bits(rb) || f32_bits(qa) != f32_bits(qb);
  return bad;
}

/* order-independent digest of the four f64 results (wrapping sum over all inputs) */
TRIG_FN uint64_t trig_digest(double s0, double c0, double s1, double c1) {
  uint64_t a, b, c, d;
  memcpy(&a, &s0, 8); memcpy(&b, &c0, 8); memcpy(&c, &s1, 8); memcpy(&d, &c1, 8);
  return a + 3 * b + 5 * c + 7 * d;
}
