/* pyrandom.c — ORACLE / TEST INFRASTRUCTURE ONLY (see pyrandom.h). */
#include "pyrandom.h"

#define MT_N 624
#define MT_M 397
#define MATRIX_A 0x9908b0dfU
#define UPPER_MASK 0x80000000U
#define LOWER_MASK 0x7fffffffU

static void init_genrand(pyrandom* r, uint32_t s) {
  uint32_t* mt = r->mt;
  mt[0] = s;
  int i;
  for (i = 1; i < MT_N; i++) mt[i] = (1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i);
  r->index = i;
}

static void init_by_array(pyrandom* r, const uint32_t* key, int key_length) {
  uint32_t* mt = r->mt;
  init_genrand(r, 19650218U);
  int i = 1, j = 0;
  int k = (MT_N > key_length ? MT_N : key_length);
  for (; k; k--) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
    i++;
    j++;
    if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
    if (j >= key_length) j = 0;
  }
  for (k = MT_N - 1; k; k--) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
    i++;
    if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
  }
  mt[0] = 0x80000000U;
}

void pyrandom_seed(pyrandom* r, uint64_t seed) {
  uint32_t key[2];
  int n;
  key[0] = (uint32_t)(seed & 0xffffffffU);
  key[1] = (uint32_t)(seed >> 32);
  n = key[1] ? 2 : 1; /* 32-bit chunks of abs(seed); seed 0 -> one zero word */
  init_by_array(r, key, n);
}

uint32_t pyrandom_u32(pyrandom* r) {
  static const uint32_t mag01[2] = {0x0U, MATRIX_A};
  uint32_t* mt = r->mt;
  uint32_t y;
  if (r->index >= MT_N) {
    int kk;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
      y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
      mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 0x1U];
    }
    for (; kk < MT_N - 1; kk++) {
      y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
      mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 0x1U];
    }
    y = (mt[MT_N - 1] & UPPER_MASK) | (mt[0] & LOWER_MASK);
    mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 0x1U];
    r->index = 0;
  }
  y = mt[r->index++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680U;
  y ^= (y << 15) & 0xefc60000U;
  y ^= (y >> 18);
  return y;
}

double pyrandom_random(pyrandom* r) {
  uint32_t a = pyrandom_u32(r) >> 5, b = pyrandom_u32(r) >> 6;
  return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

double pyrandom_uniform(pyrandom* r, double a, double b) { return a + (b - a) * pyrandom_random(r); }
