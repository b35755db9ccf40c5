// tdm_step_wg.hip — TDM.step (gym_macm/envs/combat.py:104-184) for 64 < N <= 4096 agents per env:
// the reference takes any team sizes (combat.py:82-83) in an uncapped b2World (cm_framework.py:161);
// the wave kernel (flock_step_w64.hip, env_step_w64<kTdm>) holds one agent per lane, N <= 64.
//
// One workgroup per env, one thread per agent (blockDim = N rounded up to 64); above 1024 agents 1024
// threads with 2 or 4 agents each (round 5: the pair records then in HBM):
//   1. the action loop (combat.py:121-155) exactly as the wave kernel's: rotation (f32
//      SetTransform), force with the movement penalty, cooldowns, and the melee ray casts. Bodies do
//      not move during the loop and deaths come after it, so every cast sees the same world and all
//      rays are cast in parallel (candidates in body order, b2CircleShape::RayCast clipping the
//      fraction, as the oracle's b2l_world_raycast); only the shared listener's updates and the
//      damage are applied in agent order, by thread 0;
//   2. deaths (combat.py:157-165); the combat state is committed to HBM;
//   3. the physics, TDM.get_obs, done / winner by the spill step (flock_spill.hpp, MODE kTdm): the
//      touching-contact working set in HBM, the per-body arrays and pair records in LDS (88 B per
//      body: 88 KB at N = 1024), the observation in memory order (tdm_obs_block_linear).
// The spill step's arithmetic and order are those of the fast kernels, so results are bit-exact
// against the oracle (tests/test_gpu_tdm_wg.py). HBM per agent-step is dominated by the [N, N-1, 4]
// observation (16 (N-1) B at float32), as in the wave kernel.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include "flock_common.hpp"
#include "tdm_obs.hpp"
#include "flock_spill.hpp"

namespace macm {
namespace tdmwg {

constexpr int W = 64;

__host__ __device__ constexpr int a16(int x) { return (x + 15) & ~15; }
__host__ __device__ constexpr int words(int N) { return (N + 31) / 32; }

// LDS of the action loop (dead when the spill step starts; it reuses the same bytes)
struct PreLayout {
  int c, hp, hit, aw, atw, total;
};
__host__ __device__ constexpr PreLayout pre_layout(int N) {
  PreLayout L{};
  int o = 0;
  L.c = o;  o = a16(o + 8 * N);            // float2 positions
  L.hp = o; o = a16(o + 8 * N);            // f64 health (damage applied in agent order)
  L.hit = o; o = a16(o + 4 * N);           // int32 ray hit of each attacker (-1: none)
  L.aw = o; o = a16(o + 4 * words(N));     // bitmap: alive at the step's start
  L.atw = o; o = a16(o + 4 * words(N));    // bitmap: attacking this step
  L.total = o;
  return L;
}

// the init / observe kernels' LDS: positions, angles, alive bitmap, fat AABBs, scan scratch
struct ObsLayout {
  int c, a, aw, fat, scan, total;
};
__host__ __device__ constexpr ObsLayout obs_layout(int N) {
  ObsLayout L{};
  int o = 0;
  L.c = o;  o = a16(o + 8 * N);
  L.a = o;  o = a16(o + 4 * N);
  L.aw = o; o = a16(o + 4 * words(N));
  L.fat = o; o = a16(o + 16 * N);
  L.scan = o; o = a16(o + 4 * 32);
  L.total = o;
  return L;
}

// wave w's ballot of body chunk j (bodies j BS + 64w ..) -> words 2 (j BS / 64 + w), + 1 of an LDS
// bitmap of N bits (call with the whole block)
__device__ __forceinline__ void ballot_bits(uint32_t* bits, int N, bool v, int j = 0) {
  const unsigned long long m = __ballot(v);
  const int tid = threadIdx.x;
  if ((tid & (W - 1)) == 0) {
    const int q = 2 * ((tid + j * (int)blockDim.x) / W);
    if (q < words(N)) bits[q] = (uint32_t)m;
    if (q + 1 < words(N)) bits[q + 1] = (uint32_t)(m >> 32);
  }
}

}  // namespace tdmwg

int tdm_wg_step_lds(int N) {
  // N > 1024 (BPT > 1): the pair records in HBM (spill step RECS_LDS = false)
  const int a = tdmwg::pre_layout(N).total, b = spill::layout(N, N <= 1024).total;
  return a > b ? a : b;
}
int tdm_wg_obs_lds(int N) { return tdmwg::obs_layout(N).total; }

// BPT bodies per thread (round 5: N up to 4096 with 1024 threads; thread t holds t, t + BS, ...); BPT = 1
// with blockDim = N rounded up to 64 below 1024 agents. Every ordered step (the listener and damage in
// agent order on thread 0, the spill step's scans) sees the bodies in agent order either way.
template <typename OT, int BPT = 1>
__global__ __launch_bounds__(1024) void tdm_step_wg(StepParams P, WorldBuffers B, TdmParams TP, TdmBuffers TB,
                                                    int cur, const uchar4* __restrict__ actions,
                                                    OT* __restrict__ obs, uint8_t* __restrict__ done_out) {
  using namespace tdmwg;
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x, tid = threadIdx.x, BS = blockDim.x, N = P.n_agents;
  const PreLayout L = pre_layout(N);
  float2* s_c = (float2*)(lds + L.c);
  double* s_hpd = (double*)(lds + L.hp);
  int* s_hit = (int*)(lds + L.hit);
  uint32_t* s_aw = (uint32_t*)(lds + L.aw);
  uint32_t* s_atw = (uint32_t*)(lds + L.atw);

  // The spill working-set slot is taken before anything of this step is committed: a pool that
  // stays full (~1 s) leaves the env wholly unstepped and reported, never half-stepped
  __shared__ int s_slot;
  const int slot = spill::acquire_slot(B, e, &s_slot);
  if (slot < 0) {
    spill::keep_lists(P, B, e, cur);
    if (tid == 0) {
      B.status[e] |= MACM_ST_SPILL_WAIT;
      report_status(B, MACM_ST_SPILL_WAIT);
    }
    return;
  }
  bool act[BPT], act0[BPT], attacking[BPT];
  float2 p[BPT], F[BPT];
  float ang[BPT], ray_x[BPT], ray_y[BPT];
  double hp[BPT], cda[BPT], cdm[BPT];  // Agent.health, cooldown_atk, cooldown_mov_penalty
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    const size_t ag = (size_t)e * N + i;
    act[j] = false;
    p[j] = F[j] = make_float2(0.0f, 0.0f);
    ang[j] = ray_x[j] = ray_y[j] = 0.0f;
    hp[j] = cda[j] = cdm[j] = 0.0;
    attacking[j] = false;
    int a0 = 1, a1 = 1, a2 = 1, a3 = 0;
    if (i < N) {
      p[j] = B.pos[ag];
      ang[j] = B.angle[ag];
      const uchar4 a = actions[ag];
      a0 = a.x;
      a1 = a.y;
      a2 = a.z;
      a3 = a.w;
      act[j] = TB.alive[ag] != 0;
      hp[j] = TB.health[ag];
      cda[j] = TB.cd_atk[ag];
      cdm[j] = TB.cd_mov[ag];
      s_c[i] = p[j];
      s_hpd[i] = hp[j];
    }
    act0[j] = act[j];  // alive when the step starts (acts this step)

    // ---- the action loop (combat.py:121-155), as env_step_w64<kTdm> ------------------------------
    if (act[j]) {
      // agent.body.angle = angle + (a2-1) * rotation_speed * (1/hz) -> SetTransform(float32)
      float af = (float)((double)ang[j] + ((double)(a2 - 1) * P.rot_step) * P.inv_hz);
      const double ad = (double)af;
      if (fabs(ad) > M_PI) af = (float)(ad - sgn(ad) * (2.0 * M_PI));
      ang[j] = af;
      const double cc = ((a0 != 1) && (a1 != 1)) ? P.diag_c : 1.0;
      const double k0 = (double)(a0 - 1), k1 = (double)(a1 - 1);
      // Agent.force = _force * (1 - percent_mov_penalty * int(cooldown_mov_penalty > 0))   combat.py:46-49
      const double force = P.force * (1.0 - TP.percent_mov_penalty * (double)(cdm[j] > 0.0));
      double s0, c0, s1, c1;  // np.cos / np.sin of angle and angle + pi/2
      act_trig(af, &s0, &c0, &s1, &c1);
      F[j].x = 0.0f + (float)((c0 * k0 + c1 * k1) * cc * force);  // ApplyForce onto ClearForces' zero
      F[j].y = 0.0f + (float)((s0 * k0 + s1 * k1) * cc * force);
      if (cda[j] <= 0.0) {
        if (a3) {
          attacking[j] = true;
          // point2 = point1 + (range*cos(angle), range*sin(angle)): a float32 add of the
          // float32-converted tuple
          ray_x[j] = p[j].x + (float)(TP.melee_range * c0);
          ray_y[j] = p[j].y + (float)(TP.melee_range * s0);
          cda[j] = TP.cooldown_atk;
          cdm[j] = TP.cooldown_mov_penalty;
        }
      } else {
        cda[j] -= P.inv_hz;
        if (TP.decay_mov_penalty) cdm[j] -= P.inv_hz;
      }
    }
    ballot_bits(s_aw, N, act[j], j);
    ballot_bits(s_atw, N, attacking[j], j);
  }
  __syncthreads();  // positions, health and both bitmaps visible

  // ---- ray casts: b2World::RayCast + RayCastClosestCallback (cm_framework.py:56-86) --------------
#pragma unroll
  for (int jj = 0; jj < BPT; ++jj) {
    if (!attacking[jj]) continue;
    int hit = -1;
    const float rvx = ray_x[jj] - p[jj].x, rvy = ray_y[jj] - p[jj].y;  // r = p2 - p1
    const float rrr = rvx * rvx + rvy * rvy;
    const float rad2 = P.radius * P.radius;
    float maxf = 1.0f;
    for (int q = 0; q < words(N); ++q)
      for (uint32_t m = s_aw[q]; m; m &= m - 1u) {
        const int j = 32 * q + __builtin_ctz(m);
        const float2 cj = s_c[j];
        const float sx = p[jj].x - cj.x, sy = p[jj].y - cj.y;  // s = p1 - position
        const float bb = (sx * sx + sy * sy) - rad2;
        const float c = sx * rvx + sy * rvy;
        const float sigma = c * c - rrr * bb;
        if (sigma < 0.0f || rrr < kEps) continue;
        float a = -(c + sqrtf(sigma));
        if (0.0f <= a && a <= maxf * rrr) {
          a /= rrr;
          maxf = a;
          hit = j;
        }
      }
    s_hit[tid + jj * BS] = hit;
  }
  __syncthreads();
  int2 lis = make_int2(0, -1);
  if (tid == 0) {
    // listener.hit / listener.fixture persist across casts and steps (literal), or reset per cast
    // (fresh_raycast); damage in agent order (combat.py:152-153)
    lis = TB.listener[e];
    for (int q = 0; q < words(N); ++q)
      for (uint32_t m = s_atw[q]; m; m &= m - 1u) {
        const int h = s_hit[32 * q + __builtin_ctz(m)];
        if (TP.fresh_raycast) {
          if (h >= 0) s_hpd[h] -= TP.melee_dmg;
        } else {
          if (h >= 0) lis = make_int2(1, h);
          if (lis.x) s_hpd[lis.y] -= TP.melee_dmg;
        }
      }
  }
  __syncthreads();
  int n_alive0 = 0, n_att = 0, n_died = 0;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    if (i < N) hp[j] = s_hpd[i];
    if (act[j] && hp[j] <= 0.0) act[j] = false;  // deaths: body.active = False (combat.py:157-165)
    n_alive0 += __syncthreads_count(act0[j]);
    n_att += __syncthreads_count(attacking[j]);
    n_died += __syncthreads_count(act0[j] && !act[j]);
  }

  // ---- commit the combat state (the spill step reads it back) ------------------------------------
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    const size_t ag = (size_t)e * N + i;
    if (i < N) {
      if (act0[j]) {
        B.angle[ag] = ang[j];
        TB.cd_atk[ag] = cda[j];
        TB.cd_mov[ag] = cdm[j];
      }
      TB.health[ag] = hp[j];
      TB.alive[ag] = act[j] ? 1 : 0;
      if (TB.health_out) TB.health_out[ag] = hp[j];
      if (TB.alive_out) TB.alive_out[ag] = act[j] ? 1 : 0;
    }
  }
  if (tid == 0) {
    TB.listener[e] = lis;
    unsigned long long* ec = B.env_counters + (size_t)e * 4;
    ec[0] += (unsigned long long)n_alive0;
    ec[1] += (unsigned long long)n_att;
    ec[2] += (unsigned long long)n_died;
  }
  __threadfence_block();
  // ---- Box2D step of the living bodies, TDM.get_obs, done / winner --------------------------------
  // (above 1024 agents the pair records live in the slot's HBM: 48 B per body would not fit beside
  // the per-body arrays)
  spill::step_env<OT, BPT == 1, kTdm, BPT, true>(P, B, e, cur, actions, obs, nullptr, nullptr, nullptr, done_out, lds, &TP,
                                           &TB, F, slot);
}

// TDM world creation (combat.py:78-102) for N > 64: every body active with init_health, zero
// cooldowns, the fresh listener, fat AABBs and the first FindNewContacts list (every overlapping
// pair, a descending then b descending, as flock_init_wg), and the initial observation. The bodies in
// a loop (any N, any block size).
template <typename OT>
__global__ __launch_bounds__(1024) void tdm_init_wg(StepParams P, WorldBuffers B, TdmParams TP, TdmBuffers TB,
                                                    int cur, OT* __restrict__ obs, const uint8_t* __restrict__ mask) {
  using namespace tdmwg;
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x, tid = threadIdx.x, BS = blockDim.x, N = P.n_agents, C = P.max_contacts;
  if (mask && !mask[e]) return;  // reset_envs: only the masked envs
  const ObsLayout L = obs_layout(N);
  float2* s_c = (float2*)(lds + L.c);
  float* s_a = (float*)(lds + L.a);
  uint32_t* s_aw = (uint32_t*)(lds + L.aw);
  float4* s_f = (float4*)(lds + L.fat);
  int* s_scan = (int*)(lds + L.scan);
  for (int i = tid; i < N; i += BS) {
    const size_t ag = (size_t)e * N + i;
    const float2 p = B.pos[ag];
    const float r = P.radius;
    const float4 f = make_float4((p.x - r) - kAabbExtension, (p.y - r) - kAabbExtension, (p.x + r) + kAabbExtension,
                                 (p.y + r) + kAabbExtension);
    B.fat[ag] = f;
    B.vel[ag] = make_float2(0.0f, 0.0f);
    B.sleep[ag] = 0.0f;
    TB.health[ag] = TP.init_health;
    TB.cd_atk[ag] = 0.0;
    TB.cd_mov[ag] = 0.0;
    TB.alive[ag] = 1;
    if (TB.health_out) TB.health_out[ag] = TP.init_health;
    if (TB.alive_out) TB.alive_out[ag] = 1;
    s_c[i] = p;
    s_a[i] = B.angle[ag];
    s_f[i] = f;
  }
  for (int q = tid; q < words(N); q += BS) s_aw[q] = q + 1 < words(N) || N % 32 == 0 ? ~0u : (1u << (N % 32)) - 1u;
  __syncthreads();
  // pairs in (a desc, b desc) order: chunks of BS bodies in body order, the total first
  int total = 0;
  for (int i0 = 0; i0 < N; i0 += BS) {
    const int i = i0 + tid;
    int cnt = 0;
    if (i < N)
      for (int j = i + 1; j < N; ++j) cnt += spill::overlap(s_f[i], s_f[j]) ? 1 : 0;
    int excl;
    total += spill::block_scan_excl(cnt, excl, s_scan);
  }
  int base = 0;
  for (int i0 = 0; i0 < N; i0 += BS) {
    const int i = i0 + tid;
    int cnt = 0;
    if (i < N)
      for (int j = i + 1; j < N; ++j) cnt += spill::overlap(s_f[i], s_f[j]) ? 1 : 0;
    int excl;
    const int tot = spill::block_scan_excl(cnt, excl, s_scan);
    if (i < N && cnt > 0) {
      int w = total - (base + excl) - cnt;  // agents > i come first
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
  const size_t rows = (size_t)e * N * (N - 1);
  for (int i = tid; i - tid < N; i += BS)  // tdm_obs_block returns for i >= N
    tdm_obs_block<OT>(obs ? obs + rows * 4 : nullptr, TB.mask_out ? TB.mask_out + rows : nullptr, N, i, s_aw, TP,
                      s_c, s_a);
  if (tid == 0) {
    const int st = total > C ? MACM_ST_CONTACT_OVERFLOW : 0;
    B.ccount[cur][e] = total > C ? C : total;
    B.step_count[e] = 0;
    B.time_passed[e] = 0.0;
    B.done[e] = 0;
    B.status[e] = st;
    if (st) report_status(B, st);
    TB.listener[e] = make_int2(0, -1);
    TB.winner[e] = -1;
    if (TB.winner_out) TB.winner_out[e] = -1;
  }
}

// TDM.get_obs of the current state without stepping (N > 64; the bodies in a loop).
template <typename OT>
__global__ __launch_bounds__(1024) void tdm_observe_wg(StepParams P, WorldBuffers B, TdmParams TP, TdmBuffers TB,
                                                       OT* __restrict__ obs) {
  using namespace tdmwg;
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x, tid = threadIdx.x, BS = blockDim.x, N = P.n_agents;
  const ObsLayout L = obs_layout(N);
  float2* s_c = (float2*)(lds + L.c);
  float* s_a = (float*)(lds + L.a);
  uint32_t* s_aw = (uint32_t*)(lds + L.aw);
  for (int i0 = 0, j = 0; i0 < N; i0 += BS, ++j) {
    const int i = i0 + tid;
    const size_t ag = (size_t)e * N + i;
    bool live = false;
    if (i < N) {
      s_c[i] = B.pos[ag];
      s_a[i] = B.angle[ag];
      live = TB.alive[ag] != 0;
    }
    ballot_bits(s_aw, N, live, j);
  }
  __syncthreads();
  const size_t rows = (size_t)e * N * (N - 1);
  for (int i = tid; i - tid < N; i += BS)
    tdm_obs_block<OT>(obs ? obs + rows * 4 : nullptr, TB.mask_out ? TB.mask_out + rows : nullptr, N, i, s_aw, TP,
                      s_c, s_a);
}

// ---- host-side launchers (C++ linkage, used by macm_capi.hip) -------------------------------------
static int tdm_wg_block(int N) { return N > 1024 ? 1024 : ((N + 63) / 64) * 64; }

// as wg_configure: the kernels' dynamic-LDS limits only grow (per device)
hipError_t tdm_wg_configure(int N) {
  static std::mutex mu;
  static std::map<int, int> high;
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  int& hw = high[dev];
  if (N <= hw) return hipSuccess;
  hw = N;
  const int ls = tdm_wg_step_lds(N), lo = tdm_wg_obs_lds(N);
  const void* fs[] = {(const void*)tdm_step_wg<float>, (const void*)tdm_step_wg<double>,
                      (const void*)tdm_step_wg<float, 2>, (const void*)tdm_step_wg<double, 2>,
                      (const void*)tdm_step_wg<float, 4>, (const void*)tdm_step_wg<double, 4>};
  const void* fo[] = {(const void*)tdm_init_wg<float>, (const void*)tdm_init_wg<double>,
                      (const void*)tdm_observe_wg<float>, (const void*)tdm_observe_wg<double>};
  hipError_t e = hipSuccess;
  for (const void* f : fs)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, ls);
  for (const void* f : fo)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lo);
  return e;
}

hipError_t launch_tdm_step_wg(const StepParams& P, const WorldBuffers& B, const TdmParams& TP, const TdmBuffers& TB,
                              int cur, const void* actions, void* obs, bool obs_f64, uint8_t* done, hipStream_t s) {
  const dim3 grid(P.n_envs), block(tdm_wg_block(P.n_agents));
  const int lds = tdm_wg_step_lds(P.n_agents);
  const int bpt = P.n_agents <= 1024 ? 1 : P.n_agents <= 2048 ? 2 : 4;
  const uchar4* a = (const uchar4*)actions;
  if (obs_f64) {
    if (bpt == 1) hipLaunchKernelGGL((tdm_step_wg<double, 1>), grid, block, lds, s, P, B, TP, TB, cur, a, (double*)obs, done);
    else if (bpt == 2) hipLaunchKernelGGL((tdm_step_wg<double, 2>), grid, block, lds, s, P, B, TP, TB, cur, a, (double*)obs, done);
    else hipLaunchKernelGGL((tdm_step_wg<double, 4>), grid, block, lds, s, P, B, TP, TB, cur, a, (double*)obs, done);
  } else {
    if (bpt == 1) hipLaunchKernelGGL((tdm_step_wg<float, 1>), grid, block, lds, s, P, B, TP, TB, cur, a, (float*)obs, done);
    else if (bpt == 2) hipLaunchKernelGGL((tdm_step_wg<float, 2>), grid, block, lds, s, P, B, TP, TB, cur, a, (float*)obs, done);
    else hipLaunchKernelGGL((tdm_step_wg<float, 4>), grid, block, lds, s, P, B, TP, TB, cur, a, (float*)obs, done);
  }
  return hipGetLastError();
}

hipError_t launch_tdm_init_wg(const StepParams& P, const WorldBuffers& B, const TdmParams& TP, const TdmBuffers& TB,
                              int cur, void* obs, bool obs_f64, const uint8_t* mask, hipStream_t s) {
  const dim3 grid(P.n_envs), block(tdm_wg_block(P.n_agents));
  const int lds = tdm_wg_obs_lds(P.n_agents);
  if (obs_f64)
    hipLaunchKernelGGL(tdm_init_wg<double>, grid, block, lds, s, P, B, TP, TB, cur, (double*)obs, mask);
  else
    hipLaunchKernelGGL(tdm_init_wg<float>, grid, block, lds, s, P, B, TP, TB, cur, (float*)obs, mask);
  return hipGetLastError();
}

hipError_t launch_tdm_observe_wg(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                                 const TdmBuffers& TB, void* obs, bool obs_f64, hipStream_t s) {
  const dim3 grid(P.n_envs), block(tdm_wg_block(P.n_agents));
  const int lds = tdm_wg_obs_lds(P.n_agents);
  if (obs_f64)
    hipLaunchKernelGGL(tdm_observe_wg<double>, grid, block, lds, s, P, B, TP, TB, (double*)obs);
  else
    hipLaunchKernelGGL(tdm_observe_wg<float>, grid, block, lds, s, P, B, TP, TB, (float*)obs);
  return hipGetLastError();
}

}  // namespace macm
