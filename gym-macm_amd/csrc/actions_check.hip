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

// set_state's contact lists (macm_world_set_state), checked on the device (a host loop
// over E x C entries): the kernels index a list by its count and its packed pairs, so every env
// needs 0 <= count <= C and a < b < N in each of its first `count` entries. One block per env; the
// lowest failing (env << 32 | entry) is kept, entry 0xffffffff for a count out of range.
// C: row pitch of ab; cap: entries of a row that hold the caller's list (min(C, the caller's stride))
__global__ void check_lists_kernel(const int32_t* __restrict__ count, const uint32_t* __restrict__ ab, int C, int cap,
                                   int N, unsigned long long* __restrict__ first_bad) {
  const int e = blockIdx.x;
  const int n = count[e];
  if (n < 0 || n > cap) {
    if (threadIdx.x == 0) atomicMin(first_bad, ((unsigned long long)e << 32) | 0xffffffffull);
    return;
  }
  const uint32_t* row = ab + (size_t)e * C;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const uint32_t v = row[k], a = v & 0xffffu, b = v >> 16;
    if (!(a < b && b < (uint32_t)N)) atomicMin(first_bad, ((unsigned long long)e << 32) | (unsigned)k);
  }
}

hipError_t launch_check_lists(const int32_t* count, const uint32_t* ab, int E, int C, int cap, int N,
                              unsigned long long* first_bad, hipStream_t s) {
  hipLaunchKernelGGL(check_lists_kernel, dim3((unsigned)E), dim3(256), 0, s, count, ab, C, cap, N, first_bad);
  return hipGetLastError();
}

}  // namespace macm
