/* tools/trig_check.c — exhaustive check of macm_sincos (gym-macm_amd/csrc/macm_math.h,
 * the same source the kernels compile) against glibc sin/cos, which the reference's
 * math.cos/math.sin call (mvmnt.py:113-116, combat.py:147).
 *
 * The action path evaluates sin/cos at ad = (double)angle_f32 and at ad + pi/2 (f64 sum),
 * so the inputs are exactly the float32 values: every one with |x| < 2^19 (both signs)
 * is checked. For any input where an f64 result differs, the float32 quantities the step
 * derives from it are compared too: the forces f32((c0*k0 + c1*k1)*cc*F) and
 * f32((s0*k0 + s1*k1)*cc*F) for k0,k1 in {-1,0,1}, cc in {1, 1/sqrt(2)}, F in {20, 16}
 * (Flock, TDM with the move penalty), and the melee ray offsets f32(2*c0), f32(2*s0).
 *
 *   gcc -O2 -fopenmp -ffp-contract=off -I gym-macm_amd/csrc -I tools tools/trig_check.c -lm -o /tmp/trig_check
 *   /tmp/trig_check [--ocml gpurun_out/trig/ocml_records.bin]   (about 30 s on 8 cores)
 *   /tmp/trig_check --stride 61     every 61st input (tests/test_action_trig.py)
 *   /tmp/trig_check --raw --emit gym-macm_amd/csrc/trig_fix.inc   regenerate the exception table
 * The --ocml records come from tools/trig_gpu_check.hip on the GPU (device libm).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "macm_math.h"
#include "trig_outcomes.h"

static uint64_t bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

struct Rec { uint32_t xbits, pad; double s0, c0, s1, c1; };  /* tools/trig_gpu_check.hip */

static void glibc_at(uint32_t u, double* s0, double* c0, double* s1, double* c1) {
  float f; memcpy(&f, &u, 4);
  const double x = (double)f, x1 = x + M_PI / 2;
  *s0 = sin(x); *c0 = cos(x); *s1 = sin(x1); *c1 = cos(x1);
}

static int in_pi(uint32_t u) { float f; memcpy(&f, &u, 4); return fabs((double)f) <= M_PI + 0.1; }

int main(int argc, char** argv) {
  const char* ocml = NULL;
  const char* emit = NULL;
  int raw = 0;
  long long stride = 1;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--raw")) raw = 1;
    else if (!strcmp(argv[i], "--ocml") && i + 1 < argc) ocml = argv[++i];
    else if (!strcmp(argv[i], "--emit") && i + 1 < argc) emit = argv[++i];
    else if (!strcmp(argv[i], "--stride") && i + 1 < argc) stride = atoll(argv[++i]);
    else { fprintf(stderr, "usage: %s [--stride S] [--raw [--emit trig_fix.inc]] [--ocml FILE]\n", argv[0]); return 2; }
  }
  if (stride != 1 && (emit || ocml)) { fprintf(stderr, "--emit / --ocml need the full set (stride 1)\n"); return 2;
  }
  const uint32_t lim = 0x49000000u;  /* 2^19 as float32 bits */
  long long n = 0, mis[4] = {0}, mis_pi[4] = {0}, f32bad = 0, f32bad_pi = 0;
  uint64_t dig = 0;
  static uint32_t bad[4096];
  int nbad = 0;
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : n, f32bad, f32bad_pi, dig) \
    reduction(+ : mis[:4], mis_pi[:4])
  for (long long k = 0; k < 2LL * lim; k += stride) {
    const uint32_t u = (uint32_t)(k < lim ? k : (k - lim) | 0x80000000u);
    float f; memcpy(&f, &u, 4);
    const double x = (double)f, x1 = x + M_PI / 2;
    double s0m, c0m, s1m, c1m;
    if (raw) {
      macm_action_trig_raw(x, &s0m, &c0m, &s1m, &c1m);
    } else {
      macm_action_trig(f, &s0m, &c0m, &s1m, &c1m);
    }
    dig += trig_digest(s0m, c0m, s1m, c1m);
    const double s0g = sin(x), c0g = cos(x), s1g = sin(x1), c1g = cos(x1);
    const int d[4] = {bits(s0m) != bits(s0g), bits(c0m) != bits(c0g),
                      bits(s1m) != bits(s1g), bits(c1m) != bits(c1g)};
    const int p = in_pi(u);
    ++n;
    for (int i = 0; i < 4; ++i) { mis[i] += d[i]; if (p) mis_pi[i] += d[i]; }
    if (d[0] | d[1] | d[2] | d[3]) {
      const int b = f32_outcomes_differ(c0m, s0m, c1m, s1m, c0g, s0g, c1g, s1g);
      f32bad += b;
      if (p) f32bad_pi += b;
      if (b) {
#pragma omp critical
        {
          if (nbad < 4096) bad[nbad++] = u;
          printf("%s: float32 outcome differs at x=%a (%.9g)\n", raw ? "macm_action_trig_raw" : "macm_action_trig", x, x);
        }
      }
    }
  }
  printf("inputs: %lld float32 values, |x| < 2^19 (stride %lld)\n", n, stride);
  printf("host %s digest %016llx\n", raw ? "macm_action_trig_raw" : "macm_action_trig", (unsigned long long)dig);
  printf("%s f64 mismatches vs glibc  sin(x) %lld  cos(x) %lld  sin(x+pi/2) %lld  cos(x+pi/2) %lld\n",
         raw ? "macm_action_trig_raw" : "macm_action_trig", mis[0], mis[1], mis[2], mis[3]);
  printf("  of which |x| <= pi+0.1: %lld %lld %lld %lld\n", mis_pi[0], mis_pi[1], mis_pi[2], mis_pi[3]);
  printf("%s: inputs whose float32 forces / ray offsets differ from glibc's: %lld (|x| <= pi+0.1: %lld)\n",
         raw ? "macm_action_trig_raw" : "macm_action_trig", f32bad, f32bad_pi);
  if (raw && emit) {  /* the exception table for macm_math.h: glibc's values at these inputs */
    for (int i = 1; i < nbad; ++i)
      for (int j = i; j > 0 && bad[j - 1] > bad[j]; --j) { uint32_t t = bad[j]; bad[j] = bad[j - 1]; bad[j - 1] = t; }
    FILE* fo = fopen(emit, "w");
    if (!fo) { perror(emit); return 2; }
    fprintf(fo, "// Generated by tools/trig_check.c --raw --emit: the float32 angles a where macm_action_trig_raw's\n"
                "// derived float32 forces / melee-ray offsets differ from glibc's, with glibc's\n"
                "// sin(a), cos(a), sin(a + pi/2), cos(a + pi/2) (see macm_action_trig).\n");
    for (int far = 0; far < 2; ++far) {
      int cnt = 0;
      for (int i = 0; i < nbad; ++i) { float f; memcpy(&f, &bad[i], 4); cnt += (fabsf(f) >= 4.0f) == far; }
      fprintf(fo, "#define MACM_TRIG_N%s %d\n", far ? "FAR" : "NEAR", cnt);
      fprintf(fo, "MACM_MATH_TABLE double kTrigFix%s[%d][5] = {\n", far ? "Far" : "Near", cnt ? cnt : 1);
      if (!cnt) fprintf(fo, "    {1e30, 0, 0, 0, 0},\n");
      for (int i = 0; i < nbad; ++i) {
        double s0, c0, s1, c1;
        float f; memcpy(&f, &bad[i], 4);
        if ((fabsf(f) >= 4.0f) != far) continue;
        glibc_at(bad[i], &s0, &c0, &s1, &c1);
        fprintf(fo, "    {%af, %a, %a, %a, %a},\n", (double)f, s0, c0, s1, c1);
      }
      fprintf(fo, "};\n");
    }
    fclose(fo);
    printf("wrote %s (%d entries)\n", emit, nbad);
  }
  if (ocml) {
    /* D_ocml = (D_mine minus R) + {x in R : ocml outcome != glibc outcome}, where R is the
       set of inputs at which ocml's and macm_sincos's outcomes differ (device records). */
    FILE* fp = fopen(ocml, "rb");
    if (!fp) { perror(ocml); return 2; }
    uint32_t nr = 0;
    if (fread(&nr, 4, 1, fp) != 1) return 2;
    struct Rec* r = malloc(sizeof(struct Rec) * (nr ? nr : 1));
    if (fread(r, sizeof(struct Rec), nr, fp) != nr) return 2;
    fclose(fp);
    long long dl = 0, dl_pi = 0;
    for (int i = 0; i < nbad; ++i) {
      int inR = 0;
      for (uint32_t j = 0; j < nr; ++j) inR |= r[j].xbits == bad[i];
      if (!inR) { ++dl; dl_pi += in_pi(bad[i]); }
    }
    for (uint32_t j = 0; j < nr; ++j) {
      double s0, c0, s1, c1;
      glibc_at(r[j].xbits, &s0, &c0, &s1, &c1);
      if (f32_outcomes_differ(r[j].c0, r[j].s0, r[j].c1, r[j].s1, c0, s0, c1, s1)) {
        float f; memcpy(&f, &r[j].xbits, 4);
        printf("ocml: float32 outcome differs at x=%a (%.9g)\n", (double)f, (double)f);
        ++dl; dl_pi += in_pi(r[j].xbits);
      }
    }
    printf("ocml (device libm, %u device records): inputs whose float32 forces / ray offsets differ from glibc's: %lld (|x| <= pi+0.1: %lld)\n",
           nr, dl, dl_pi);
    free(r);
  }
  return f32bad != 0;
}
