// tdm_obs_snap.hip — the split TDM observation (round 6).
//
// TDM.get_obs (gym_macm/envs/combat.py:206-227) is O(N^2) float64 work per env (at 2 x 16: 496 pairs,
// an atan2 core each, and 992 16-B slots), which the wave kernel runs on its one wave after the
// physics: 55% of a wave's cycles at C4 (tools/tdm_phase.py). With one wave per env and fewer envs
// than SIMDs (C4's per-GPU shard: 512 envs over 1,024 SIMDs) that work waits on one wave's latency.
// In the split form the step writes only each agent's pose after the step (TdmBuffers::snap_out:
// x, y, angle, alive; 16 B) and this kernel observes every (step, env) row with a workgroup of its
// own: 256 threads stage one atan2 core and distance per unordered pair in LDS, then write the
// slots in memory order (whole 128-B lines, the mask as 256 consecutive bytes per store).
//
// Every value is bit-identical to the wave kernel's pair form (tdm_obs.hpp tdm_obs_pair_m): the
// same float32 rel per direction, the shared atan2 core of |rel| (|xj - xi| == |xi - xj| in IEEE
// arithmetic), each direction's own quadrant, "- angle" and wrap, p = wrap(aj - ai), r =
// obs_sqrt<OT> of the same float32 distance.
#include "flock_common.hpp"
#include "tdm_obs.hpp"

namespace macm {

constexpr int kSnapBlock = 256;

// the stage: per unordered pair (i < j, row-major) its atan2 core and r, both double
__host__ __device__ constexpr int tdm_snap_stage_bytes(int N) { return 16 * (N * (N - 1) / 2); }

// first pair index of row i (pairs (i, j > i) row-major)
__device__ __forceinline__ int pair_start(int N, int i) { return (i * (2 * N - i - 1)) >> 1; }

template <typename OT>
__global__ __launch_bounds__(kSnapBlock) void tdm_observe_snap(TdmParams TP, int N, const float4* __restrict__ snap,
                                                               OT* __restrict__ obs, uint8_t* __restrict__ mask) {
  extern __shared__ __align__(16) unsigned char lds[];
  __shared__ float2 s_c[64];
  __shared__ float s_a[64];
  __shared__ unsigned long long s_live;
  const size_t row = blockIdx.x;  // (step, env) row of the snapshot [rows, N]
  const int tid = threadIdx.x, BS = blockDim.x;
  const int S = N - 1, P = N * S / 2;
  if (tid < 64) {
    const float4 q = tid < N ? snap[row * N + tid] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    s_c[tid] = make_float2(q.x, q.y);
    s_a[tid] = q.z;
    const unsigned long long live = __ballot(tid < N && q.w != 0.0f);
    if (tid == 0) s_live = live;
  }
  __syncthreads();
  const unsigned long long livem = s_live;
  double* const s_core = reinterpret_cast<double*>(lds);
  double* const s_r = s_core + P;
  // pass 1: one unordered pair per thread, its shared part
  for (int p = tid; p < P; p += BS) {
    const float b = (float)(2 * N - 1);
    int i = (int)((b - sqrtf(b * b - 8.0f * (float)p)) * 0.5f);
    i = i < 0 ? 0 : (i > N - 2 ? N - 2 : i);
    while (i > 0 && pair_start(N, i) > p) --i;
    while (i < N - 2 && pair_start(N, i + 1) <= p) ++i;
    const int j = p - pair_start(N, i) + i + 1;
    if ((livem >> i) & (livem >> j) & 1ull) {
      const float2 ci = s_c[i], cj = s_c[j];
      const float rx = cj.x - ci.x, ry = cj.y - ci.y;
      s_r[p] = obs_sqrt<OT>(rx * rx + ry * ry);
      s_core[p] = obs_atan2_core(fabs((double)rx), fabs((double)ry));
    }
  }
  __syncthreads();
  // pass 2: slot q = i * S + k of the row's [N, N-1] block, other agent j = k < i ? k : k + 1
  OT* const o = obs ? obs + row * (size_t)N * S * 4 : nullptr;
  uint8_t* const m = mask ? mask + row * (size_t)N * S : nullptr;
  const int ns = N * S;
  for (int q = tid; q < ns; q += BS) {
    const int i = q / S, k = q - i * S;
    const int j = k < i ? k : k + 1;
    const bool live = ((livem >> i) & (livem >> j) & 1ull) != 0ull;
    double r = 0.0, t = 0.0, pr = 0.0, ty = 0.0;
    if (live) {
      const int pp = i < j ? pair_start(N, i) + (j - i - 1) : pair_start(N, j) + (i - j - 1);
      const float2 ci = s_c[i], cj = s_c[j];
      const float rx = cj.x - ci.x, ry = cj.y - ci.y;  // other.position - agent.position
      r = s_r[pp];
      t = wrap_pi(obs_atan2_finish(s_core[pp], (double)ry, (double)rx) - (double)s_a[i]);
      pr = wrap_pi((double)s_a[j] - (double)s_a[i]);
      ty = tdm_team_nb(TP, j) == tdm_team_nb(TP, i) ? 1.0 : 0.0;
    }
    if (o) store4<OT>(o + (size_t)q * 4, r, t, pr, ty);
    if (m) m[q] = live ? 1 : 0;
  }
}

// rows (step, env) of snapshots -> their observation rows (obs [rows, N, N-1, 4], mask [rows, N, N-1])
hipError_t launch_tdm_observe_snap(const TdmParams& TP, int N, size_t rows, const float4* snap, void* obs,
                                   bool obs_f64, uint8_t* mask, hipStream_t s) {
  if (rows == 0 || (!obs && !mask)) return hipSuccess;
  if (N < 2 || N > 64) return hipErrorInvalidValue;
  const int lds = tdm_snap_stage_bytes(N);
  if (obs_f64)
    hipLaunchKernelGGL(tdm_observe_snap<double>, dim3((unsigned)rows), dim3(kSnapBlock), lds, s, TP, N, snap,
                       (double*)obs, mask);
  else
    hipLaunchKernelGGL(tdm_observe_snap<float>, dim3((unsigned)rows), dim3(kSnapBlock), lds, s, TP, N, snap,
                       (float*)obs, mask);
  return hipGetLastError();
}

}  // namespace macm
