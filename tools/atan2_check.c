/* tools/atan2_check.c — accuracy check of the observation atan2 (csrc/macm_math.h
 * obs_atan2, the same source compiled for the host) against glibc atan2 on float32-valued inputs:
 * ulp histogram, and whether "atan2 - angle" rounded to float32 ever differs.
 *   gcc -O2 -ffp-contract=off -I gym-macm_amd/csrc tools/atan2_check.c -lm -o /tmp/atan2_check && /tmp/atan2_check */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include "macm_math.h"
/* the observation atan2 the kernels compile (csrc/macm_math.h) */
static double fa_atan2(double y, double x) { return obs_atan2(y, x); }
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
