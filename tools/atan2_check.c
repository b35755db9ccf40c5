/* tools/atan2_check.c — accuracy check of the observation atan2 (csrc/flock_common.hpp
 * obs_atan2, same formulas in C with fma) against glibc atan2 on float32-valued inputs:
 * ulp histogram, and whether "atan2 - angle" rounded to float32 ever differs.
 *   gcc -O2 -ffp-contract=off tools/atan2_check.c -lm -o /tmp/atan2_check && /tmp/atan2_check */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
static const double aT[] = {
  3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01,
 -1.11111104054623557880e-01, 9.09088713343650656196e-02, -7.69187620504482999495e-02,
  6.66107313738753120669e-02, -5.83357013379057348645e-02, 4.97687799461593236017e-02,
 -3.65315727442169155270e-02, 1.62858201153657823623e-02};
static const double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
/* GPU form: selects, fma Horner in z (single chain), one reduction division */
double fa_atan2(double y, double x) {
  double ax = fabs(x), ay = fabs(y);
  double mx = ax > ay ? ax : ay, mn = ax > ay ? ay : ax;
  int swap = ay > ax;
  /* reduction of a = mn/mx in [0,1] without forming a: ids -1, 0, 1 (a <= 1 < 1.1875);
     thresholds 7/16 and 11/16 times mx are exact */
  double c_a, c_b, c_c, c_d, hi, lo; int id;  /* c_c == c_a */
  if (mn < 0.4375 * mx) { id = -1; c_a = 1; c_b = 0; c_c = 1; c_d = 0; hi = 0; lo = 0; }
  else if (mn < 0.6875 * mx) { id = 0; c_a = 2; c_b = 1; c_c = 2; c_d = 1; hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
  else { id = 1; c_a = 1; c_b = 1; c_c = 1; c_d = 1; hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
  double xr = fma(c_a, mn, -c_b * mx) / fma(c_d, mn, c_c * mx);
  double z = xr * xr;
  double p = aT[10];
  for (int k = 9; k >= 0; --k) p = fma(p, z, aT[k]);
  double s = z * p;                 /* s1 + s2 */
  double r = id < 0 ? fma(-xr, s, xr) : hi - (fma(xr, s, -lo) - xr);
  /* undo the swap: atan(ay/ax) = pi/2 - atan(ax/ay) */
  if (swap) r = (1.57079632679489655800e+00 - r) + 6.12323399573676603587e-17;
  if (x < 0) r = (pi - r) + pi_lo;
  if (mx == 0.0) r = x < 0 || signbit(x) ? pi : 0.0;
  return signbit(y) ? -r : r;
}
static int64_t ulpd(double a, double b) { int64_t ia, ib; memcpy(&ia,&a,8); memcpy(&ib,&b,8); if (ia<0) ia = INT64_MIN - ia; if (ib<0) ib = INT64_MIN - ib; return llabs(ia-ib); }
int main() {
  srand(1); int64_t maxu = 0; long cnt[8] = {0}; long n = 20000000; long f32diff = 0;
  for (long i = 0; i < n; ++i) {
    float fx = (float)(((double)rand()/RAND_MAX - 0.5) * 60), fy = (float)(((double)rand()/RAND_MAX - 0.5) * 60);
    if (i % 7 == 0) fy = fx * (float)((double)rand()/RAND_MAX * 1e-3);
    if (i % 11 == 0) fx = fy * (float)((double)rand()/RAND_MAX * 1e-3);
    double g = atan2((double)fy, (double)fx), f = fa_atan2((double)fy, (double)fx);
    int64_t u = ulpd(g, f); if (u > maxu) { maxu = u; printf("new max %lld at y=%a x=%a g=%.17g f=%.17g\n",(long long)u,(double)fy,(double)fx,g,f);} cnt[u < 7 ? u : 7]++;
    double ang = ((double)rand()/RAND_MAX - 0.5) * 6.28;  float fa = (float)ang;
    double tg = g - (double)fa, tf = f - (double)fa;
    if ((float)tg != (float)tf) f32diff++;
  }
  printf("max ulp %lld\n", (long long)maxu); for (int k = 0; k < 8; ++k) printf("%d: %ld\n", k, cnt[k]);
  printf("f32 result differs: %ld of %ld\n", f32diff, n);
  double sp[][2] = {{0,0},{-0.0,0},{0,-0.0},{-0.0,-0.0},{1,0},{-1,0},{0,1},{0,-1},{1,1},{-1,-1},{1,-1}};
  for (int k = 0; k < 11; ++k) printf("atan2(%g,%g): glibc %.17g fa %.17g\n", sp[k][0], sp[k][1], atan2(sp[k][0],sp[k][1]), fa_atan2(sp[k][0],sp[k][1]));
}
