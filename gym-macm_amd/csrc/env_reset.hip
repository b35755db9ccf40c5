// env_reset.hip — per-env episode reset on the device.
//
// The reference draws every pose from Python's global `random` (mvmnt.py:60-64,
// combat.py:83-85) and its reset() draws the next poses from the same stream
// (mvmnt.py:224-233, combat.py:234-245; the Flock one keeps the targets). Each env
// here owns the CPython MT19937 stream it was seeded with at macm_*_reset; the
// state lives in HBM ([E][kMtStride] words), so resetting the envs of a device mask
// (e.g. the done flags) continues every env's stream exactly as a reference env
// would after `random.seed(seed + e)`, with no host round trip:
//   draw_poses_kernel : MT19937 words (block-parallel twist), random() = res53,
//                       Flock x = spread*(r-0.5)+start, y likewise, angle =
//                       uniform(-1,1)*pi; TDM x = r*(team + width/2), y = r*height,
//                       angle as Flock; written to pos / angle of masked envs
//   then the env's init kernel (with the same mask) rebuilds proxies, the first
//   contact list and the initial observation.
// Every operation is integer or exactly rounded double arithmetic, so the poses
// equal the host generator's bit for bit.
#include "flock_common.hpp"

namespace macm {

constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr int kMaxDrawWords = 6 * 1024;

__device__ __forceinline__ uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ uint32_t mix(uint32_t hi, uint32_t lo, uint32_t src) {
  const uint32_t y = (hi & 0x80000000u) | (lo & 0x7fffffffu);
  return src ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// One MT19937 twist of s_mt in place, block-parallel. Sequential semantics:
// mt[k] = mix(mt[k], mt[k+1], mt[(k+397) % 624]) for k = 0..623 in order, where
// mt[k+1] is still old and mt[k+397-624] already new. Phases [0,227), [227,454),
// [454,623), {623} each read only values final for their phase.
__device__ void mt_twist(uint32_t* s_mt, int tid, int nt) {
  const int lo[4] = {0, kMtN - kMtM, 2 * (kMtN - kMtM), kMtN - 1};
  const int hi[4] = {kMtN - kMtM, 2 * (kMtN - kMtM), kMtN - 1, kMtN};
  for (int ph = 0; ph < 4; ++ph) {
    uint32_t v[4];
    int n = 0;
    for (int k = lo[ph] + tid; k < hi[ph]; k += nt) {
      const int src = k + kMtM < kMtN ? k + kMtM : k + kMtM - kMtN;
      v[n++] = mix(s_mt[k], s_mt[(k + 1) % kMtN], s_mt[src]);
    }
    __syncthreads();
    n = 0;
    for (int k = lo[ph] + tid; k < hi[ph]; k += nt) s_mt[k] = v[n++];
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void draw_poses_kernel(const uint8_t* __restrict__ mask, uint32_t* __restrict__ mt,
                                                         PoseDraw D, float2* __restrict__ pos,
                                                         float* __restrict__ angle) {
  const int e = blockIdx.x;
  if (!mask[e]) return;
  const int tid = threadIdx.x, nt = blockDim.x, N = D.n_agents;
  __shared__ uint32_t s_mt[kMtN];
  __shared__ uint32_t s_w[kMaxDrawWords];
  uint32_t* g = mt + (size_t)e * kMtStride;
  for (int k = tid; k < kMtN; k += nt) s_mt[k] = g[k];
  int idx = (int)g[kMtN];
  __syncthreads();
  // three random() per agent, two words each, in chunks of kMaxDrawWords / 6 agents (the stream's
  // words stay in draw order: chunk after chunk, agent after agent)
  constexpr int kChunk = kMaxDrawWords / 6;
  for (int i0 = 0; i0 < N; i0 += kChunk) {
    const int n = min(kChunk, N - i0);
    const int need = 6 * n;
    for (int got = 0; got < need;) {
      if (idx >= kMtN) {
        mt_twist(s_mt, tid, nt);
        idx = 0;
      }
      const int take = min(kMtN - idx, need - got);
      for (int w = tid; w < take; w += nt) s_w[got + w] = temper(s_mt[idx + w]);
      got += take;
      idx += take;
      __syncthreads();
    }
    for (int q0 = tid; q0 < n; q0 += nt) {
      const int i = i0 + q0;
      double r[3];
      for (int q = 0; q < 3; ++q) {  // random.random(): genrand_res53
        const uint32_t a = s_w[6 * q0 + 2 * q] >> 5, b = s_w[6 * q0 + 2 * q + 1] >> 6;
        r[q] = (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
      }
      double x, y;
      if (D.mode == kFlock) {  // mvmnt.py:62-63
        x = D.spread * (r[0] - 0.5) + D.start_x;
        y = D.spread * (r[1] - 0.5) + D.start_y;
      } else {  // combat.py:83-84
        x = r[0] * ((double)tdm_team_of(D.TP, i) + D.half_width);
        y = r[1] * D.height;
      }
      const double a = (-1.0 + (1.0 - -1.0) * r[2]) * M_PI;  // random.uniform(-1, 1) * np.pi
      pos[(size_t)e * N + i] = make_float2((float)x, (float)y);
      angle[(size_t)e * N + i] = (float)a;
    }
    __syncthreads();  // the chunk's words are read before the next chunk overwrites them
  }
  for (int k = tid; k < kMtN; k += nt) g[k] = s_mt[k];
  if (tid == 0) g[kMtN] = (uint32_t)idx;
}

hipError_t launch_draw_poses(const uint8_t* mask, uint32_t* mt, const PoseDraw& D, int n_envs, float2* pos,
                             float* angle, hipStream_t s) {
  hipLaunchKernelGGL(draw_poses_kernel, dim3(n_envs), dim3(256), 0, s, mask, mt, D, pos, angle);
  return hipGetLastError();
}

}  // namespace macm
