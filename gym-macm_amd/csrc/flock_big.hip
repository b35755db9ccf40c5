// flock_big.hip — Flock worlds of 1024 < N <= 4096 agents per env (round 5).
//
// The reference steps any sum(n_agents) (gym_macm/envs/mvmnt.py:61) in one uncapped b2World. The
// fast kernels hold one body per thread of one workgroup (N <= 1024); here an env is one workgroup of
// 1024 threads and each thread holds BPT = ceil(N / 1024) bodies (t, t + 1024, ...):
//   - the step is the spill step (flock_spill.hpp step_env<OT, false, kFlock, BPT>): the touching
//     contacts, their CSR edges, island order and records in the env's HBM working-set slot, the
//     per-body arrays in LDS (~38 B per body: 151 KB at N = 4096), the pair records in HBM, the
//     island DFS on thread 0 and each island's Gauss-Seidel on one thread. Same arithmetic and order
//     as every other path, so results are bit-exact against the oracle (tests/test_gpu_big.py);
//   - reset (FindNewContacts of the first step, the initial obs) and observe loop over the bodies.
// Correctness first: no BASELINE config exceeds 1024 agents (C5 is 1024), and the serial island
// walk and per-island solves of a dense 4096-body world take milliseconds per env-step.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include "flock_common.hpp"
#include "flock_spill.hpp"

namespace macm {
namespace big {

constexpr int kBS = 1024;  // threads per env

__host__ __device__ constexpr int a16(int x) { return (x + 15) & ~15; }

// init / observe LDS: positions, fat AABBs, scan scratch (24 B per body: 96 KB at N = 4096)
struct InitLayout {
  int c, f, scan, total;
};
__host__ __device__ constexpr InitLayout init_layout(int N) {
  InitLayout L{};
  int o = 0;
  L.c = o;  o = a16(o + 8 * N);
  L.f = o;  o = a16(o + 16 * N);
  L.scan = o; o = a16(o + 4 * 32);
  L.total = o;
  return L;
}

}  // namespace big

// Reset (macm_world_reset / _place / _reset_envs): fat AABBs, zeroed dynamics, the first
// FindNewContacts list (every overlapping pair, (a, b) descending) and the initial observation, as
// flock_init_wg with the bodies in a loop. mask: reset_envs' selection (NULL: every env).
template <typename OT>
__global__ __launch_bounds__(1024) void flock_init_big(StepParams P, WorldBuffers B, int cur, OT* __restrict__ obs,
                                                       int32_t* __restrict__ nbr_out, const uint8_t* __restrict__ mask) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x, tid = threadIdx.x, BS = blockDim.x, N = P.n_agents, C = P.max_contacts;
  if (mask && !mask[e]) return;
  const big::InitLayout L = big::init_layout(N);
  float2* s_c = (float2*)(lds + L.c);
  float4* s_f = (float4*)(lds + L.f);
  int* s_scan = (int*)(lds + L.scan);
  const float r = P.radius;
  for (int i = tid; i < N; i += BS) {
    const size_t ag = (size_t)e * N + i;
    const float2 p = B.pos[ag];
    const float4 f = make_float4((p.x - r) - kAabbExtension, (p.y - r) - kAabbExtension, (p.x + r) + kAabbExtension,
                                 (p.y + r) + kAabbExtension);
    B.fat[ag] = f;
    B.vel[ag] = make_float2(0.0f, 0.0f);
    B.sleep[ag] = 0.0f;
    s_c[i] = p;
    s_f[i] = f;
  }
  __syncthreads();
  // pairs (a, b > a) in descending order: body a's block of its pairs starts at the number of pairs
  // of the bodies above it; chunks of BS bodies in body order, each a block scan
  int base = 0, total = 0;
  for (int i0 = 0; i0 < N; i0 += BS) {  // the total first: the list's start of body a needs it
    const int i = i0 + tid;
    int cnt = 0;
    if (i < N)
      for (int j = i + 1; j < N; ++j) cnt += spill::overlap(s_f[i], s_f[j]) ? 1 : 0;
    int excl;
    total += spill::block_scan_excl(cnt, excl, s_scan);
  }
  for (int i0 = 0; i0 < N; i0 += BS) {
    const int i = i0 + tid;
    int cnt = 0;
    if (i < N)
      for (int j = i + 1; j < N; ++j) cnt += spill::overlap(s_f[i], s_f[j]) ? 1 : 0;
    int excl;
    const int tot = spill::block_scan_excl(cnt, excl, s_scan);
    if (i < N && cnt > 0) {
      int w = total - (base + excl) - cnt;
      for (int j = N - 1; j > i; --j)
        if (spill::overlap(s_f[i], s_f[j])) {
          if (w < C) {
            B.cab[cur][(size_t)e * C + w] = (uint32_t)i | ((uint32_t)j << 16);
            B.cimp[cur][(size_t)e * C + w] = make_float2(0.0f, 0.0f);
          }
          ++w;
        }
    }
    base += tot;
  }
  for (int i = tid; i < N; i += BS) {
    const size_t ag = (size_t)e * N + i;
    const float2 p = s_c[i];
    float best = __builtin_inff();
    int bj = i == 0 ? 1 : 0;
    for (int j = 0; j < N; ++j) {
      const float2 q = s_c[j];
      const float dx = q.x - p.x, dy = q.y - p.y;
      const float d2 = dx * dx + dy * dy;
      if (j != i && d2 < best) {  // strict '<': the lowest index wins ties
        best = d2;
        bj = j;
      }
    }
    if (nbr_out) nbr_out[ag] = bj;
    if (obs) {
      const float2 tg = B.targets[(size_t)e * P.n_targets + B.tidx[i]];
      const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
      const float tdx = tg.x - p.x, tdy = tg.y - p.y;
      const float2 cb = s_c[bj];
      spill::write_obs<OT>(obs + ag * od, P.coord, B.angle[ag], best, cb.x - p.x, cb.y - p.y, tdx, tdy,
                           tdx * tdx + tdy * tdy);
    }
  }
  if (tid == 0) {
    B.ccount[cur][e] = total > C ? C : total;
    B.step_count[e] = 0;
    B.time_passed[e] = 0.0;
    B.done[e] = 0;
    B.status[e] = total > C ? MACM_ST_CONTACT_OVERFLOW : 0;
    if (total > C) report_status(B, MACM_ST_CONTACT_OVERFLOW);
  }
}

// Flock.get_obs of the current state (macm_world_observe)
template <typename OT>
__global__ __launch_bounds__(1024) void flock_observe_big(StepParams P, WorldBuffers B, OT* __restrict__ obs,
                                                          int32_t* __restrict__ nbr_out) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x, tid = threadIdx.x, BS = blockDim.x, N = P.n_agents;
  float2* s_c = (float2*)lds;
  for (int i = tid; i < N; i += BS) s_c[i] = B.pos[(size_t)e * N + i];
  __syncthreads();
  for (int i = tid; i < N; i += BS) {
    const size_t ag = (size_t)e * N + i;
    const float2 p = s_c[i];
    float best = __builtin_inff();
    int bj = i == 0 ? 1 : 0;
    for (int j = 0; j < N; ++j) {
      const float2 q = s_c[j];
      const float dx = q.x - p.x, dy = q.y - p.y;
      const float d2 = dx * dx + dy * dy;
      if (j != i && d2 < best) {
        best = d2;
        bj = j;
      }
    }
    if (nbr_out) nbr_out[ag] = bj;
    if (obs) {
      const float2 tg = B.targets[(size_t)e * P.n_targets + B.tidx[i]];
      const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
      const float tdx = tg.x - p.x, tdy = tg.y - p.y;
      const float2 cb = s_c[bj];
      spill::write_obs<OT>(obs + ag * od, P.coord, B.angle[ag], best, cb.x - p.x, cb.y - p.y, tdx, tdy,
                           tdx * tdx + tdy * tdy);
    }
  }
}

// One env.step of env blockIdx.x: the spill step with BPT bodies per thread
template <typename OT, int BPT>
__global__ __launch_bounds__(1024) void flock_step_big(StepParams P, WorldBuffers B, int cur,
                                                       const void* __restrict__ actions, OT* __restrict__ obs,
                                                       int32_t* __restrict__ nbr_out, float* __restrict__ rew_out,
                                                       uint8_t* __restrict__ coll_out, uint8_t* __restrict__ done_out) {
  extern __shared__ __align__(16) unsigned char lds[];
  spill::step_env<OT, false, kFlock, BPT>(P, B, blockIdx.x, cur, actions, obs, nbr_out, rew_out, coll_out, done_out,
                                          lds);
}

int big_step_lds(int N) { return spill::layout(N, false).total; }
int big_init_lds(int N) { return big::init_layout(N).total; }

// Dynamic LDS limits of the big kernels (the largest N configured per device, as wg_configure)
hipError_t big_configure(int N) {
  static std::mutex mu;
  static std::map<int, int> high;
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  int& hw = high[dev];
  if (N <= hw) return hipSuccess;
  hw = N;
  hipError_t e = hipSuccess;
  const int ls = big_step_lds(N), li = big_init_lds(N), lo = 8 * N;
  const void* fs[] = {(const void*)flock_step_big<float, 2>, (const void*)flock_step_big<double, 2>,
                      (const void*)flock_step_big<float, 4>, (const void*)flock_step_big<double, 4>};
  for (const void* f : fs)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, ls);
  const void* fi[] = {(const void*)flock_init_big<float>, (const void*)flock_init_big<double>};
  for (const void* f : fi)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, li);
  const void* fo[] = {(const void*)flock_observe_big<float>, (const void*)flock_observe_big<double>};
  for (const void* f : fo)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lo);
  return e;
}

hipError_t launch_step_big(const StepParams& P, const WorldBuffers& B, int cur, const void* actions, void* obs,
                           bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done, hipStream_t s) {
  const dim3 grid(P.n_envs), block(big::kBS);
  const int lds = big_step_lds(P.n_agents);
  const bool four = P.n_agents > 2 * big::kBS;
  if (obs_f64) {
    if (four)
      hipLaunchKernelGGL((flock_step_big<double, 4>), grid, block, lds, s, P, B, cur, actions, (double*)obs, nbr, rew,
                         coll, done);
    else
      hipLaunchKernelGGL((flock_step_big<double, 2>), grid, block, lds, s, P, B, cur, actions, (double*)obs, nbr, rew,
                         coll, done);
  } else {
    if (four)
      hipLaunchKernelGGL((flock_step_big<float, 4>), grid, block, lds, s, P, B, cur, actions, (float*)obs, nbr, rew,
                         coll, done);
    else
      hipLaunchKernelGGL((flock_step_big<float, 2>), grid, block, lds, s, P, B, cur, actions, (float*)obs, nbr, rew,
                         coll, done);
  }
  return hipGetLastError();
}

hipError_t launch_init_big(const StepParams& P, const WorldBuffers& B, int cur, void* obs, bool obs_f64, int32_t* nbr,
                           const uint8_t* mask, hipStream_t s) {
  const dim3 grid(P.n_envs), block(big::kBS);
  const int lds = big_init_lds(P.n_agents);
  if (obs_f64)
    hipLaunchKernelGGL(flock_init_big<double>, grid, block, lds, s, P, B, cur, (double*)obs, nbr, mask);
  else
    hipLaunchKernelGGL(flock_init_big<float>, grid, block, lds, s, P, B, cur, (float*)obs, nbr, mask);
  return hipGetLastError();
}

hipError_t launch_observe_big(const StepParams& P, const WorldBuffers& B, void* obs, bool obs_f64, int32_t* nbr,
                              hipStream_t s) {
  const dim3 grid(P.n_envs), block(big::kBS);
  const int lds = 8 * P.n_agents;
  if (obs_f64)
    hipLaunchKernelGGL(flock_observe_big<double>, grid, block, lds, s, P, B, (double*)obs, nbr);
  else
    hipLaunchKernelGGL(flock_observe_big<float>, grid, block, lds, s, P, B, (float*)obs, nbr);
  return hipGetLastError();
}

}  // namespace macm
