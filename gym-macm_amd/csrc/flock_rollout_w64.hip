// Multi-step wave kernels (macm_world_rollout / macm_tdm_rollout): the step body of
// flock_step_w64.hip inside a loop over steps, compiled as its own translation unit with
// -mllvm -disable-machine-licm (see the rollout section of flock_step_w64.hip and the Makefile).
#define MACM_ROLLOUT_TU 1
#include "flock_step_w64.hip"
