// bots.hip — the reference's scripted actors on the device (test_scripts/bots.py),
// reading the step kernels' observation tensors and writing the next actions, so
// closed-loop rollouts never leave HBM.
// The decisions themselves are in bots.hpp (shared with the closed-loop rollout).
#include "bots.hpp"

namespace macm {

template <typename OT>
__global__ __launch_bounds__(256) void bots_flock_kernel(const OT* __restrict__ obs, int od, long long rows,
                                                         uint8_t* __restrict__ act) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  bot_flock_row(obs + i * od, od, act + i * 3);
}

template <typename OT>
__global__ __launch_bounds__(256) void bots_combat_kernel(const OT* __restrict__ obs, const uint8_t* __restrict__ mask,
                                                          int N, long long rows, uint8_t* __restrict__ act) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  bot_combat_row(obs + i * (N - 1) * 4, mask + i * (N - 1), N, act + i * 4);
}

hipError_t launch_bots_flock(const void* obs, bool obs_f64, int od, long long rows, uint8_t* act, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int B = 256;
  const dim3 grid((unsigned)((rows + B - 1) / B));
  if (obs_f64)
    hipLaunchKernelGGL(bots_flock_kernel<double>, grid, dim3(B), 0, s, (const double*)obs, od, rows, act);
  else
    hipLaunchKernelGGL(bots_flock_kernel<float>, grid, dim3(B), 0, s, (const float*)obs, od, rows, act);
  return hipGetLastError();
}

hipError_t launch_bots_combat(const void* obs, const uint8_t* mask, bool obs_f64, int N, long long rows,
                              uint8_t* act, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int B = 256;
  const dim3 grid((unsigned)((rows + B - 1) / B));
  if (obs_f64)
    hipLaunchKernelGGL(bots_combat_kernel<double>, grid, dim3(B), 0, s, (const double*)obs, mask, N, rows, act);
  else
    hipLaunchKernelGGL(bots_combat_kernel<float>, grid, dim3(B), 0, s, (const float*)obs, mask, N, rows, act);
  return hipGetLastError();
}

}  // namespace macm
