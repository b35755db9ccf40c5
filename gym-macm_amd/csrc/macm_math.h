// macm_math.h — the f64 elementary functions the step evaluates itself instead of
// calling the device libm. One source for both sides: the HIP kernels include it, and
// the host checks (tools/trig_check.c, tools/atan2_check.c) compile the SAME code with
// gcc -ffp-contract=off and compare it with glibc, which is what the reference's
// math.cos / math.sin / math.atan2 / np.arctan2 call. Every operation is a single IEEE
// op (fma only where written), so host and device results are bit-identical.
#pragma once
#include <math.h>

#ifdef __HIPCC__
#define MACM_MATH_FN __device__ __forceinline__
#else
#define MACM_MATH_FN static inline
#endif

// sin and cos of one argument, |x| < 2^19 * pi/2 (beyond that: the library, see the
// caller). Cody-Waite reduction x = n*pi/2 + (y0 + y1) with pi/2 split into 33-bit
// pieces p1 + p2 + p2t (fdlibm e_rem_pio2.c's constants): n*p1 and n*p2 are exact for
// |n| < 2^20, x - n*p1 is exact, and the second subtraction keeps its rounding error
// (Fast2Sum: the minuend is a multiple of the subtrahend's ulp), so the remainder carries
// ~119 bits of pi/2 with no data-dependent branch (enough for every float32 input: the
// exhaustive check below). Then the fdlibm
// minimax kernels (k_sin.c / k_cos.c) on the double-double remainder, Horner in fma.
// Exhaustively compared with glibc sin/cos on every float32-valued x in range and on
// x + pi/2 (tools/trig_check.c; result in DESIGN.md §3).
MACM_MATH_FN void macm_sincos(double x, double* sp, double* cp) {
  const double fn = rint(x * 6.36619772367581382433e-01);  // round(x * 2/pi)
  const int q = (int)fn;
  const double t1 = fma(-fn, 1.57079632673412561417e+00, x);  // exact
  const double w2 = fn * 6.07710050630396597660e-11;            // exact
  const double r2 = t1 - w2;
  const double e2 = (t1 - r2) - w2;
  const double tail = fma(-fn, 2.02226624879595063154e-21, e2);  // pio2_2t
  const double y0 = r2 + tail;
  const double y1 = (r2 - y0) + tail;
  const double z = y0 * y0;
  // k_sin: sin(y0 + y1) = y0 + (y0^3 S(z) + y1 (1 - z/2) ...)
  double ps = 1.58969099521155010221e-10;
  ps = fma(ps, z, -2.50507602534068634195e-08);
  ps = fma(ps, z, 2.75573137070700676789e-06);
  ps = fma(ps, z, -1.98412698298579493134e-04);
  ps = fma(ps, z, 8.33333333332248946124e-03);
  const double v = z * y0;
  const double s = y0 - ((z * (0.5 * y1 - v * ps) - y1) - v * -1.66666666666666324348e-01);
  // k_cos: cos(y0 + y1) = 1 - z/2 + z^2 C(z) - y0*y1, with the 1 - z/2 split exact
  double pc = -1.13596475577881948265e-11;
  pc = fma(pc, z, 2.08757232129817482790e-09);
  pc = fma(pc, z, -2.75573143513906633035e-07);
  pc = fma(pc, z, 2.48015872894767294178e-05);
  pc = fma(pc, z, -1.38888888888741095749e-03);
  pc = fma(pc, z, 4.16666666666666019037e-02);
  const double hz = 0.5 * z;
  const double wc = 1.0 - hz;
  const double c = wc + (((1.0 - wc) - hz) + (z * (z * pc) - y0 * y1));
  const int odd = q & 1;
  double so = odd ? c : s, co = odd ? s : c;
  if (q & 2) so = -so;
  if ((q + 1) & 2) co = -co;
  *sp = (x == 0.0) ? x : so;  // sin(-0) = -0
  *cp = co;
}

// sin/cos of x and of x1 = fl64(x + pi/2) (the reference's `angle + np.pi/2`) from ONE
// reduction. With P = fl64(pi/2) = pi/2 - c (c = 6.123e-17) and x1 = x + P - err (err the
// rounding error of the sum, exact by TwoSum), x1 - (q+1) pi/2 = (y0 + y1) - (c + err):
// the second argument has the same leading remainder y0 (so the same z and the same
// minimax polynomials) and the correction y1' = y1 - (c + err), a first-order term of both
// kernels like y1; |err| <= ulp(x1)/2, so this is only accurate for small |x| (|x| < 4:
// |y1'| < 2^-51; see macm_action_trig_raw). Its quadrant is q + 1. The kernels are then
// finished twice: ~30 f64 ops instead of a second full evaluation.
MACM_MATH_FN void macm_sincos_pair(double x, double* s0p, double* c0p, double* s1p, double* c1p) {
  const double fn = rint(x * 6.36619772367581382433e-01);  // round(x * 2/pi)
  const int q = (int)fn;
  const double t1 = fma(-fn, 1.57079632673412561417e+00, x);  // exact
  const double w2 = fn * 6.07710050630396597660e-11;            // exact
  const double r2 = t1 - w2;
  const double e2 = (t1 - r2) - w2;
  const double tail = fma(-fn, 2.02226624879595063154e-21, e2);  // pio2_2t
  const double y0 = r2 + tail;
  const double y1 = (r2 - y0) + tail;
  // x1 = x + P and its rounding error err = (x + P) - x1 (TwoSum)
  const double P = 1.57079632679489655800e+00;
  const double x1 = x + P;
  const double bp = x1 - x;
  const double err = (x - (x1 - bp)) + (P - bp);
  const double y1b = y1 - (6.12323399573676603587e-17 + err);
  const double z = y0 * y0;
  double ps = 1.58969099521155010221e-10;
  ps = fma(ps, z, -2.50507602534068634195e-08);
  ps = fma(ps, z, 2.75573137070700676789e-06);
  ps = fma(ps, z, -1.98412698298579493134e-04);
  ps = fma(ps, z, 8.33333333332248946124e-03);
  const double v = z * y0;
  const double vs = v * -1.66666666666666324348e-01;
  const double vps = v * ps;
  const double sa = y0 - ((z * (0.5 * y1 - vps) - y1) - vs);
  const double sb = y0 - ((z * (0.5 * y1b - vps) - y1b) - vs);
  double pc = -1.13596475577881948265e-11;
  pc = fma(pc, z, 2.08757232129817482790e-09);
  pc = fma(pc, z, -2.75573143513906633035e-07);
  pc = fma(pc, z, 2.48015872894767294178e-05);
  pc = fma(pc, z, -1.38888888888741095749e-03);
  pc = fma(pc, z, 4.16666666666666019037e-02);
  const double hz = 0.5 * z;
  const double wc = 1.0 - hz;
  const double cz = ((1.0 - wc) - hz) + z * (z * pc);
  const double ca = wc + (cz - y0 * y1);
  const double cb = wc + (cz - y0 * y1b);
  // quadrant q: (sin, cos) = (sa, ca) rotated; quadrant q + 1 for x1
  const int odd = q & 1;
  double so = odd ? ca : sa, co = odd ? sa : ca;
  if (q & 2) so = -so;
  if ((q + 1) & 2) co = -co;
  const int q1 = q + 1;
  double so1 = odd ? sb : cb, co1 = odd ? cb : sb;  // (q1 & 1) == !odd
  if (q1 & 2) so1 = -so1;
  if ((q1 + 1) & 2) co1 = -co1;
  *s0p = (x == 0.0) ? x : so;  // sin(-0) = -0
  *c0p = co;
  *s1p = so1;
  *c1p = co1;
}

// The action trig (mvmnt.py:113-116, combat.py:147): sin/cos of the float32 angle a and
// of a + pi/2 (an f64 sum), from which the step derives the float32 forces
// f32((c0*k0 + c1*k1)*cc*F), f32((s0*k0 + s1*k1)*cc*F) and the melee-ray offsets
// f32(range*c0), f32(range*s0). tools/trig_check.c enumerates every float32 a with
// |a| < 2^19: macm_sincos gives the same float32 quantities as glibc (the reference's
// math.cos / math.sin) for all of them (F = 20 and 16, cc = 1 and 1/sqrt(2), every
// k0, k1, range 2) except the inputs in trig_fix.inc, where glibc's values are substituted.
// With the table the derived quantities are identical to the reference's for every such
// angle; the device libm (ocml) differs at 19 of them.
#ifdef __cplusplus
#define MACM_MATH_TABLE static constexpr
#else
#define MACM_MATH_TABLE static const
#endif
#include "trig_fix.inc"  // kTrigFixNear (|a| < 4), kTrigFixFar

// The action trig before the exception table. The pair form treats the rounding error of
// x + pi/2 as a first-order correction, which is accurate only while that error is far
// below ulp(y0): |x| < 4 covers every angle the step produces (it wraps into [-pi, pi]);
// larger angles (injected state) take two independent reductions.
MACM_MATH_FN void macm_action_trig_raw(double x, double* s0, double* c0, double* s1, double* c1) {
  if (fabs(x) < 4.0) {
    macm_sincos_pair(x, s0, c0, s1, c1);
  } else {
    macm_sincos(x, s0, c0);
    macm_sincos(x + M_PI / 2, s1, c1);
  }
}

MACM_MATH_FN void macm_action_trig(float a, double* s0, double* c0, double* s1, double* c1) {
  macm_action_trig_raw((double)a, s0, c0, s1, c1);
  int hit = 0;
  for (int i = 0; i < MACM_TRIG_NNEAR; ++i) hit |= a == (float)kTrigFixNear[i][0];
  if (hit) {
    for (int i = 0; i < MACM_TRIG_NNEAR; ++i) {
      if (a == (float)kTrigFixNear[i][0]) {
        *s0 = kTrigFixNear[i][1]; *c0 = kTrigFixNear[i][2]; *s1 = kTrigFixNear[i][3]; *c1 = kTrigFixNear[i][4];
      }
    }
  }
  if (fabsf(a) >= 4.0f) {  // the step keeps angles in [-pi, pi]; larger ones come from injected state
    for (int i = 0; i < MACM_TRIG_NFAR; ++i) {
      if (a == (float)kTrigFixFar[i][0]) {
        *s0 = kTrigFixFar[i][1]; *c0 = kTrigFixFar[i][2]; *s1 = kTrigFixFar[i][3]; *c1 = kTrigFixFar[i][4];
      }
    }
  }
}

// atan2 for the observations (combat.py:221; mvmnt.py:197-198, 210-211). fdlibm's
// atan reduction (e_atan2.c / s_atan.c) with the quotient folded into one division:
// a = min(|x|,|y|) / max(|x|,|y|) is reduced by the selected (c_a*a - c_b)/(c_d*a + c_c)
// without forming a (the 7/16 and 11/16 thresholds scale max exactly), an
// 11-term Horner polynomial in FMA, then the octant/quadrant fix-ups with the split
// constants (hi + lo). Measured against glibc atan2 on 2e7 float32-valued inputs:
// <= 1 ulp, and identical after the observation's "- angle" and float32 rounding
// (tools/atan2_check.c). About half the instructions of the general library atan2.
// Split in two so that the pair (y, x) / (-y, -x) seen from both agents of a TDM pair shares
// the reduction and polynomial: obs_atan2_core depends on |x|, |y| only; obs_atan2_finish
// applies the quadrant from the signs. obs_atan2(y, x) is exactly finish(core(|x|, |y|), y, x).
MACM_MATH_FN double obs_atan2_core(double ax, double ay) {
  const int swap = ay > ax;
  const double mx = swap ? ay : ax, mn = swap ? ax : ay;
  const int r0 = mn < 0.4375 * mx;         // id -1: atan(a) directly
  const int r1 = !r0 && mn < 0.6875 * mx;  // id 0: atan(1/2) + atan((2a-1)/(2+a)); else id 1: pi/4 + ...
  const double ca = r1 ? 2.0 : 1.0, cb = r0 ? 0.0 : 1.0, cd = r0 ? 0.0 : 1.0;
  const double xr = fma(ca, mn, -(cb * mx)) / fma(cd, mn, ca * mx);
  const double z = xr * xr;
  double p = 1.62858201153657823623e-02;
  p = fma(p, z, -3.65315727442169155270e-02);
  p = fma(p, z, 4.97687799461593236017e-02);
  p = fma(p, z, -5.83357013379057348645e-02);
  p = fma(p, z, 6.66107313738753120669e-02);
  p = fma(p, z, -7.69187620504482999495e-02);
  p = fma(p, z, 9.09088713343650656196e-02);
  p = fma(p, z, -1.11111104054623557880e-01);
  p = fma(p, z, 1.42857142725034663711e-01);
  p = fma(p, z, -1.99999999998764832476e-01);
  p = fma(p, z, 3.33333333333329318027e-01);
  const double sz = z * p;
  const double hi = r1 ? 4.63647609000806093515e-01 : 7.85398163397448278999e-01;
  const double lo = r1 ? 2.26987774529616870924e-17 : 3.06161699786838301793e-17;
  double r = r0 ? fma(-xr, sz, xr) : hi - (fma(xr, sz, -lo) - xr);
  if (swap) r = (1.57079632679489655800e+00 - r) + 6.12323399573676603587e-17;
  return r;
}

MACM_MATH_FN double obs_atan2_finish(double r, double y, double x) {
  if (x < 0.0) r = (3.1415926535897931160e+00 - r) + 1.2246467991473531772e-16;
  if (x == 0.0 && y == 0.0) r = signbit(x) ? 3.1415926535897931160e+00 : 0.0;
  return copysign(r, y);
}

MACM_MATH_FN double obs_atan2(double y, double x) { return obs_atan2_finish(obs_atan2_core(fabs(x), fabs(y)), y, x); }
