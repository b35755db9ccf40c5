// actions_check.hip — the opt-in action validation of macm_world_step / macm_tdm_step
// (macm_config.validate_actions): the reference's `assert self.action_space.contains(actions)`
// before any agent acts (gym_macm/envs/mvmnt.py:94, combat.py:118).
//
//   Flock discrete    MultiDiscrete([3,3,3])   (mvmnt.py:143-145): every byte in {0, 1, 2}
//                     (int8 -1 reads as 255 and fails, as np.int8(-1) fails contains)
//   Flock continuous  Box([-1,-1], [1,1])      (mvmnt.py:146-147): -1 <= x <= 1 (NaN fails)
//   TDM               MultiDiscrete([3,3,3,2]) (combat.py:186-188) for the alive agents only:
//                     the action space is rebuilt without the dead (create_space on a death)
//
// One thread per agent row; the lowest failing flat row index is kept (atomicMin), so the host
// can name the first offending (env, agent). Not on the hot path: it runs only when enabled.
#include "flock_common.hpp"

namespace macm {

__global__ void check_actions_kernel(const void* __restrict__ actions, int mode, const uint8_t* __restrict__ alive,
                                     long long rows, unsigned long long* __restrict__ first_bad) {
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < rows;
       r += (long long)gridDim.x * blockDim.x) {
    bool ok = true;
    if (mode == 0) {  // Flock discrete
      const uint8_t* a = (const uint8_t*)actions + r * 3;
      ok = a[0] <= 2 && a[1] <= 2 && a[2] <= 2;
    } else if (mode == 1) {  // Flock continuous
      const float2 c = ((const float2*)actions)[r];
      ok = (c.x >= -1.0f && c.x <= 1.0f) && (c.y >= -1.0f && c.y <= 1.0f);
    } else {  // TDM
      if (alive && !alive[r]) continue;
      const uchar4 a = ((const uchar4*)actions)[r];
      ok = a.x <= 2 && a.y <= 2 && a.z <= 2 && a.w <= 1;
    }
    if (!ok) atomicMin(first_bad, (unsigned long long)r);
  }
}

hipError_t launch_check_actions(const void* actions, int mode, const uint8_t* alive, long long rows,
                                unsigned long long* first_bad, hipStream_t s) {
  const int bs = 256;
  long long g = (rows + bs - 1) / bs;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(check_actions_kernel, dim3((unsigned)g), dim3(bs), 0, s, actions, mode, alive, rows, first_bad);
  return hipGetLastError();
}

}  // namespace macm
