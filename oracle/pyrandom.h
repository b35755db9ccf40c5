/*
 * pyrandom.h — ORACLE / TEST INFRASTRUCTURE ONLY.
 * CPython's `random` module generator (Modules/_randommodule.c: MT19937,
 * init_by_array seeding from the 32-bit chunks of abs(seed), random() =
 * genrand_res53). The reference draws every initial position/angle/target with
 * the global `random` module (gym_macm/envs/mvmnt.py:49-50,62-64), so
 * `random.seed(s)` + Flock(...) is reproducible through this generator.
 */
#ifndef PYRANDOM_H
#define PYRANDOM_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t mt[624];
  int index;
} pyrandom;

void pyrandom_seed(pyrandom* r, uint64_t seed);  /* random.seed(int) */
uint32_t pyrandom_u32(pyrandom* r);              /* genrand_uint32 */
double pyrandom_random(pyrandom* r);             /* random.random() */
double pyrandom_uniform(pyrandom* r, double a, double b); /* random.uniform(a, b) */

#ifdef __cplusplus
}
#endif
#endif
