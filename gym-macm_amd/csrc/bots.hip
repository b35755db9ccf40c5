// bots.hip — the reference's scripted actors on the device (test_scripts/bots.py),
// reading the step kernels' observation tensors and writing the next actions, so
// closed-loop rollouts never leave HBM.
//
//   bots.flock  (bots.py:37-61): head for the target node (node 1); idle within
//                r < 1; polar: rotation = sign(t) + 1, forward = 1 + [|t| < pi/4];
//                cartesian (3-vector nodes): rotation = sign(sin t) + 1,
//                forward = 1 + [cos t > cos(pi/4)].
//   bots.combat (bots.py:3-16): closest enemy (type 0) by r, first in list order
//                on ties; rotation = sign(t) + 1, forward = 1 + [|t| < pi/5],
//                attack = [r < 3]; idle [1, 1, 1, 0] without enemies.
//
// Decisions are taken on the obs values as stored: with float64 obs they equal the
// reference's; with float32 obs a value within one float32 ulp of a threshold
// (pi/4, pi/5, 1, 3, 0) can decide differently.
#include "flock_common.hpp"

namespace macm {

constexpr double kCosQuarterPi = 0.7071067811865476;  // np.cos(np.pi / 4)

__device__ __forceinline__ int sign_plus1(double x) { return x > 0.0 ? 2 : (x < 0.0 ? 0 : 1); }

template <typename OT>
__global__ __launch_bounds__(256) void bots_flock_kernel(const OT* __restrict__ obs, int od, long long rows,
                                                         uint8_t* __restrict__ act) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  const OT* o = obs + i * od;
  const int h = od / 2;  // target node = second half of the row
  uint8_t f = 1, r = 1;
  const double tr = (double)o[h];
  if (!(tr < 1.0)) {
    if (od == 6) {  // cartesian: [r, cos t, sin t]
      r = (uint8_t)sign_plus1((double)o[h + 2]);
      f = (double)o[h + 1] > kCosQuarterPi ? 2 : 1;
    } else {
      const double t = (double)o[h + 1];
      r = (uint8_t)sign_plus1(t);
      f = fabs(t) < (M_PI / 4) ? 2 : 1;
    }
  }
  act[i * 3 + 0] = f;
  act[i * 3 + 1] = 1;
  act[i * 3 + 2] = r;
}

template <typename OT>
__global__ __launch_bounds__(256) void bots_combat_kernel(const OT* __restrict__ obs, const uint8_t* __restrict__ mask,
                                                          int N, long long rows, uint8_t* __restrict__ act) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  const int S = N - 1;
  const OT* o = obs + i * S * 4;
  const uint8_t* m = mask + i * S;
  int best = -1;
  double br = 0.0, bt = 0.0;
  for (int k = 0; k < S; ++k) {
    if (!m[k]) continue;
    if ((double)o[k * 4 + 3] != 0.0) continue;  // ally
    const double r = (double)o[k * 4];
    if (best < 0 || r < br) {  // strict '<': first closest in list order
      best = k;
      br = r;
      bt = (double)o[k * 4 + 1];
    }
  }
  uchar4 a = make_uchar4(1, 1, 1, 0);
  if (best >= 0) {
    a.x = fabs(bt) < (M_PI / 5) ? 2 : 1;
    a.z = (uint8_t)sign_plus1(bt);
    a.w = br < 3.0 ? 1 : 0;
  }
  reinterpret_cast<uchar4*>(act)[i] = a;
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
