// bots.hpp — one agent's decision of the reference's scripted actors (test_scripts/bots.py), shared
// by the bots kernels (bots.hip) and the closed-loop rollout (flock_step_w64.hip).
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
#pragma once
#include "flock_common.hpp"

namespace macm {

constexpr double kCosQuarterPi = 0.7071067811865476;  // np.cos(np.pi / 4)

__device__ __forceinline__ int sign_plus1(double x) { return x > 0.0 ? 2 : (x < 0.0 ? 0 : 1); }

// o: the agent's obs row (od = 4 polar / 6 cartesian); act: its 3 action bytes
template <typename OT>
__device__ __forceinline__ void bot_flock_row(const OT* __restrict__ o, int od, uint8_t* __restrict__ act) {
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
  act[0] = f;
  act[1] = 1;
  act[2] = r;
}

// o: the agent's [N-1, 4] obs rows (r, t, health, ally), m: their mask; act: 4 bytes (4-aligned)
template <typename OT>
__device__ __forceinline__ void bot_combat_row(const OT* __restrict__ o, const uint8_t* __restrict__ m, int N,
                                               uint8_t* __restrict__ act) {
  const int S = N - 1;
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
  *reinterpret_cast<uchar4*>(act) = a;
}

}  // namespace macm
