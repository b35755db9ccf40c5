/* tools/trig_shim.c — host build of csrc/macm_math.h for tests/test_action_trig.py (ctypes).
 *   gcc -O2 -shared -fPIC -ffp-contract=off -I gym-macm_amd/csrc tools/trig_shim.c -lm -o LIB */
#include "macm_math.h"

void shim_sincos(double x, double* s, double* c) { macm_sincos(x, s, c); }
void shim_action_trig_raw(double x, double* out) { macm_action_trig_raw(x, &out[0], &out[1], &out[2], &out[3]); }
void shim_action_trig(float a, double* out) { macm_action_trig(a, &out[0], &out[1], &out[2], &out[3]); }
double shim_obs_atan2(double y, double x) { return obs_atan2(y, x); }
