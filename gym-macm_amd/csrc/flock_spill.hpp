// flock_spill.hpp — the spill step: one env's whole Flock env.step by one workgroup, with the
// touching-contact working set in HBM, for envs whose contacts exceed the fast kernels' LDS
// capacities (dense worlds: small start_spread, injected states).
//
// The fast kernels keep every per-contact array in LDS with fixed capacities: the wave kernel
// (flock_step_w64.hip) 256 touching contacts and 16 per body, the workgroup kernel A
// (flock_step_wg.hip) 5 x blockDim up to 4608. The reference (Box2D) has no such limits: any
// start_spread is valid (gym_macm/settings.py:119-121,143-144 -> envs/mvmnt.py:62-63). When a
// fast kernel finds, after Collide and before it has written any state, that an env's touching
// contacts do not fit, the SAME workgroup calls spill::step_env for that env and returns: the
// env is stepped from its untouched start-of-step state with the touching contacts, their CSR
// edges, the island order and the island-ordered records in per-env HBM arrays sized by the
// contact-list capacity C (touching contacts are a subset of the list, so nothing can overflow
// except the list itself). Only the per-body arrays (positions, velocities, DFS state, pair
// records) stay in LDS, about 40 B per body (+ 48 B with the pair records in LDS).
//
// The arithmetic and its order are those of the fast kernels (Box2D 2.3 order, see the header
// of flock_step_w64.hip): Collide in list order, CSR edges in list (= Box2D edge) order, island
// DFS seeded in reverse body order, Gauss-Seidel in island order, position passes with the early
// exit, sleep, SynchronizeFixtures, new pairs prepended in descending (a, b) order, rewards,
// observation. Results are bit-exact against the oracle like the fast kernels
// (tests/test_gpu_dense.py forces every env through this path too).
#pragma once

#include "flock_common.hpp"
#include "tdm_obs.hpp"

namespace macm {
namespace spill {

// The level steps' contact updates on packed (x, y) pairs, as kernel B (flock_step_wg.hip
// kWgPacked): bit-identical, contraction off.
typedef float lpf2 __attribute__((ext_vector_type(2)));


constexpr int W = 64;

// TDM above one wave: the observation in memory order (tdm_obs_block_linear: whole-line stores, an
// atan2 per slot); the pair form (tdm_obs_block: one atan2 core per pair, scattered 16-B stores) was
// slower there (profiles/r03/abtests/tdm_block_obs/).

struct __align__(16) Rec {  // per-agent pair-sweep record (48 B)
  float4 fn;               // fat AABB after SynchronizeFixtures
  float4 fo;               // fat AABB at the start of the step
  float2 c;                // final position
};

__host__ __device__ constexpr int a16(int x) { return (x + 15) & ~15; }

// LDS layout of the per-body arrays (host: size check; device: carve). 16-B aligned offsets.
struct Layout {
  int c, v, slp, deg, flags, oldc, off, todo, ib, ibod, stk, ic, isolv, scan, misc, alive, recs, total;
};

__host__ __device__ constexpr Layout layout(int N, bool recs_in_lds) {
  Layout L{};
  int o = 0;
  auto take = [&](int bytes) {
    const int r = o;
    o = a16(o + bytes);
    return r;
  };
  L.c = take(8 * N);                   // float2 positions
  L.v = take(8 * N);                   // float2 velocities
  L.slp = take(4 * N);                 // sleep clocks
  L.deg = take(4 * (N + 2));           // uint32 touching degree, then the CSR fill cursor
  L.flags = take(N);                   // uint8 sleep-now
  L.oldc = take(4 * ((N + 31) / 32));  // bitmask: agent in the old list (world.contacts before)
  L.off = take(4 * (N + 1));           // uint32 CSR offsets
  L.todo = take(8 * ((N + 63) / 64));  // bodies with edges not yet in an island
  L.ib = take(2 * (N / 2 + 2));        // uint16 island body ranges
  L.ibod = take(2 * N);                // uint16 island bodies
  L.stk = take(2 * N);                 // uint16 DFS stack
  L.ic = take(4 * (N / 2 + 2));        // uint32 island contact ranges
  L.isolv = take(N / 2 + 2);           // uint8 island position-solved
  L.scan = take(4 * 32);               // block scan scratch (<= 16 waves)
  L.misc = take(4 * 8);                // nisl, status
  // TDM above one wave (tdm_step_wg.hip): bitmap of the living bodies (one wave: a ballot mask)
  L.alive = take(N > W ? 4 * ((N + 31) / 32) : 0);
  L.recs = recs_in_lds ? take((int)sizeof(Rec) * N) : o;
  L.total = o;
  return L;
}

__device__ __forceinline__ float bmin(float a, float b) { return a < b ? a : b; }  // b2Min
__device__ __forceinline__ float bmax(float a, float b) { return a > b ? a : b; }  // b2Max
__device__ __forceinline__ float sclamp(float a, float lo, float hi) { return __builtin_amdgcn_fmed3f(a, lo, hi); }
__device__ __forceinline__ bool overlap(float4 a, float4 b) {  // b2TestOverlap
  const float d1x = b.x - a.z, d1y = b.y - a.w;
  const float d2x = a.x - b.z, d2y = a.y - b.w;
  if (d1x > 0.0f || d1y > 0.0f) return false;
  if (d2x > 0.0f || d2y > 0.0f) return false;
  return true;
}
__device__ __forceinline__ void normalize(float& x, float& y) {  // b2Vec2::Normalize
  const float len = sqrt_rn(x * x + y * y);
  if (len < kEps) return;
  const float inv = rcp_rn(len);
  x *= inv;
  y *= inv;
}

// Exclusive scan over the block in thread order; returns the block total.
__device__ __forceinline__ int block_scan_excl(int v, int& excl, int* s_scan) {
  const int tid = threadIdx.x, lane = tid & (W - 1), wid = tid / W, nw = blockDim.x / W;
  const int incl = wave_prefix_sum(v);
  if (lane == W - 1) s_scan[wid] = incl;
  __syncthreads();
  int base = 0, total = 0;
  for (int w = 0; w < nw; ++w) {
    const int s = s_scan[w];
    if (w < wid) base += s;
    total += s;
  }
  __syncthreads();
  excl = base + incl - v;
  return total;
}

// The working-set slot of env e. One slot per env (sp_pool == 0): slot e. A pool (the memory budget
// holds fewer slots than envs, macm_world_create): thread 0 takes a free slot by compare-and-swap,
// starting at e % S. A holder never waits for anything while it holds a slot (it runs its spill
// step to the end and releases), so waiting envs always progress; the wait is still bounded
// (about 1 s), after which the env is not stepped and MACM_ST_SPILL_WAIT is reported. Every access
// of a slot's arrays writes before it reads, and the release writes the holder's L2 back
// (agent-scope release), so no stale line of an earlier holder can land over a later one's data.
constexpr unsigned kSlotSpins = 1u << 17;  // x s_sleep 127 (~8k cycles): ~0.5-1 s
__device__ __forceinline__ int acquire_slot(const WorldBuffers& B, int e, int* s_slot) {
  if (B.sp_pool == 0) return e;
  if (B.sp_pool < 0) return -1;  // MACM_DEBUG_SPILL_FAIL: the pool is never free (test hook)
  if (threadIdx.x == 0) {
    const int S = B.sp_pool;
    int got = -1;
    for (unsigned it = 0; got < 0 && it < kSlotSpins; ++it) {
      for (int k = 0; k < S; ++k) {
        const int q = (e + k) % S;
        if (__hip_atomic_load(&B.sp_lock[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
            atomicCAS(&B.sp_lock[q], 0u, 1u) == 0u) {
          got = q;
          break;
        }
      }
      if (got < 0) __builtin_amdgcn_s_sleep(127);
    }
    *s_slot = got;
  }
  __syncthreads();
  return *s_slot;
}

// An env that found no free slot is not stepped (MACM_ST_SPILL_WAIT): its bodies keep their
// start-of-step state, and so must its contact list, which the next step (or step k + 1 of a
// rollout) reads from the other buffer. Copies list `cur` of env e into `cur ^ 1`; every thread of
// the block calls it (without it the env resumed from a list two steps old).
__device__ __forceinline__ void keep_lists(const StepParams& P, const WorldBuffers& B, int e, int cur) {
  const int C = P.max_contacts, nxt = cur ^ 1;
  const int M = B.ccount[cur][e];
  const size_t row = (size_t)e * C;
  for (int k = threadIdx.x; k < M; k += blockDim.x) {
    B.cab[nxt][row + k] = B.cab[cur][row + k];
    B.cimp[nxt][row + k] = B.cimp[cur][row + k];
  }
  if (threadIdx.x == 0) B.ccount[nxt][e] = M;
}

__device__ __forceinline__ void release_slot(const WorldBuffers& B, int slot) {
  if (B.sp_pool <= 0) return;
  __builtin_amdgcn_s_waitcnt(0);  // this thread's stores are done (vmcnt / lgkmcnt 0)
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the XCD's L2 written back before the slot is free
    __hip_atomic_store(&B.sp_lock[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename OT>
__device__ __forceinline__ void write_obs(OT* o, int coord, float ang, float best, float rx, float ry, float tdx,
                                          float tdy, float td2) {
  const double t0 = wrap_pi(obs_atan2((double)ry, (double)rx) - (double)ang);
  const double t1 = wrap_pi(obs_atan2((double)tdy, (double)tdx) - (double)ang);
  const double r0 = obs_sqrt<OT>(best), r1 = obs_sqrt<OT>(td2);
  if (coord == MACM_COORD_CARTESIAN) {
    o[0] = (OT)r0; o[1] = (OT)cos(t0); o[2] = (OT)sin(t0);
    o[3] = (OT)r1; o[4] = (OT)cos(t1); o[5] = (OT)sin(t1);
  } else {
    o[0] = (OT)r0; o[1] = (OT)t0; o[2] = (OT)r1; o[3] = (OT)t1;
  }
}

// One env.step of env e by the calling workgroup (blockDim.x = BS >= N, a multiple of 64; every
// thread of the block must call it). `lds` holds layout(N, RECS_LDS).total bytes; the caller's
// LDS contents are dead (a barrier on entry orders its last accesses). RECS_LDS = false keeps the
// pair records in HBM (B.sp_rec) for callers whose LDS is smaller than 88 B per body.
// MODE kTdm (TDM.step, combat.py:104-184): called by the TDM wave kernel (64 threads, dense envs) or
// the workgroup TDM step (tdm_step_wg.hip, every env of more than 64 agents) after it has taken this
// step's actions, melee casts and deaths and committed them (angles, cooldowns, health, alive
// flags, listener, counters 0-2); each thread passes its force `F`. The physics skips the bodies
// that are not alive (their contacts were destroyed with their proxies) and the env layer is TDM's:
// the body state, the [N, N-1, 4] observation, done / winner, counter 3.
constexpr int kSpillChunk = 8;  // records per HBM chunk of the spill step's serial island solves

// Diagnostic build (MACM_STAMPS): phase clocks of the worlds above 1024 agents (BPT > 1: only the spill
// step runs there), stamps 16.. of the env's row (tools/big_phases.py)
#ifdef MACM_STAMPS
#define SSTAMP(k)                                                                  \
  do {                                                                             \
    if constexpr (BPT > 1) {                                                       \
      __syncthreads();                                                             \
      if (threadIdx.x == 0) B.stamps[(size_t)e * 32 + 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    }                                                                              \
  } while (0)
#else
#define SSTAMP(k) \
  do {            \
  } while (0)
#endif

template <typename OT, bool RECS_LDS, int MODE = kFlock, int BPT = 1, bool LEVELS = (BPT > 1)>
__device__ __forceinline__ void step_env(const StepParams& P, const WorldBuffers& B, int e, int cur,
                                         const void* __restrict__ actions, OT* __restrict__ obs,
                                         int32_t* __restrict__ nbr_out, float* __restrict__ rew_out,
                                         uint8_t* __restrict__ coll_out, uint8_t* __restrict__ done_out,
                                         unsigned char* lds, const TdmParams* TP = nullptr,
                                         const TdmBuffers* TB = nullptr, const float2* F = nullptr,
                                         int held_slot = -1) {
  // BPT bodies per thread (round 5, worlds above 1024 agents: blockDim.x = 1024, N <= BPT * 1024):
  // thread t holds bodies t, t + BS, ..., t + (BPT - 1) BS; every per-body step below runs for each
  // of them in that order, and every ordered reduction (block scans in body order, the pairwise
  // reward sum) takes the chunks j = 0, 1, ... in turn, so the results are those of one thread per
  // body. BPT = 1 is the form every other caller uses.
  constexpr bool kT = MODE == kTdm;
  const int tid = threadIdx.x;
  const int BS = blockDim.x;
  const int N = P.n_agents;
  const int C = P.max_contacts;
  bool act[BPT];
  size_t ag[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    act[j] = i < N && (!kT || TB->alive[(size_t)e * N + i] != 0);  // in the physics step
    ag[j] = (size_t)e * N + i;
  }
  // TDM: the living bodies, as the one wave's ballot (N <= 64, the wave kernel's hand-over) or as an
  // LDS bitmap (N > 64, the workgroup TDM step; filled below, read after the actions' barrier)
  const unsigned long long livem = kT ? __ballot(act[0]) : ~0ull;
  const int nxt = cur ^ 1;
  const Layout L = layout(N, RECS_LDS);
  float2* s_c = (float2*)(lds + L.c);
  float2* s_v = (float2*)(lds + L.v);
  float* s_slp = (float*)(lds + L.slp);
  uint32_t* s_deg = (uint32_t*)(lds + L.deg);
  uint8_t* s_flag = (uint8_t*)(lds + L.flags);
  uint32_t* s_oldc = (uint32_t*)(lds + L.oldc);
  uint32_t* s_off = (uint32_t*)(lds + L.off);
  unsigned long long* s_todo = (unsigned long long*)(lds + L.todo);
  uint16_t* s_ib = (uint16_t*)(lds + L.ib);
  uint16_t* s_ibod = (uint16_t*)(lds + L.ibod);
  uint16_t* s_stk = (uint16_t*)(lds + L.stk);
  uint32_t* s_ic = (uint32_t*)(lds + L.ic);
  uint8_t* s_isolv = (uint8_t*)(lds + L.isolv);
  int* s_scan = (int*)(lds + L.scan);
  int* s_misc = (int*)(lds + L.misc);
  uint32_t* s_alivew = (uint32_t*)(lds + L.alive);
  __syncthreads();  // the caller's last LDS accesses are done before the arrays are reused
  const bool wide = kT && N > W;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {  // wave w's ballot of chunk j holds bodies j BS + 64w .. + 63
    const unsigned long long m = j == 0 ? livem : __ballot(act[j]);
    if (wide && (tid & (W - 1)) == 0) {
      const int q = 2 * ((tid + j * BS) / W);
      if (q < (N + 31) / 32) s_alivew[q] = (uint32_t)m;
      if (q + 1 < (N + 31) / 32) s_alivew[q + 1] = (uint32_t)(m >> 32);
    }
  }
  // both bodies of a pair take part in the physics (Flock: always)
  auto live2 = [&](int a, int b) -> bool {
    if (!kT) return true;
    if (!wide) return ((livem >> a) & (livem >> b) & 1ull) != 0ull;
    return ((s_alivew[a >> 5] >> (a & 31)) & (s_alivew[b >> 5] >> (b & 31)) & 1u) != 0u;
  };
  // the HBM working set of this env's slot, capacity C (touching contacts are a subset of the list);
  // held_slot >= 0: the caller took it before committing anything (the workgroup TDM step)
  const int slot = held_slot >= 0 ? held_slot : acquire_slot(B, e, s_misc + 7);
  if (slot < 0) {  // the pool stayed full for ~1 s: not stepped (lists included), reported
    keep_lists(P, B, e, cur);
    if (tid == 0) {
      B.status[e] |= MACM_ST_SPILL_WAIT;
      report_status(B, MACM_ST_SPILL_WAIT);
    }
    return;
  }
  Rec* recs;
  if constexpr (RECS_LDS) recs = (Rec*)(lds + L.recs);
  else recs = (Rec*)B.sp_rec + (size_t)slot * N;
  uint32_t* g_tab = B.sp_tab + (size_t)slot * C;
  uint32_t* g_adj = B.sp_adj + (size_t)slot * 2 * C;
  uint32_t* g_ord = B.sp_ord + (size_t)slot * C;
  float4* g_cst = B.sp_cst + (size_t)slot * C;
  float2* g_cim = B.sp_cim + (size_t)slot * C;
  float2* g_lam = B.sp_lam + (size_t)slot * C;

  SSTAMP(0);
  // ---- loads ------------------------------------------------------------------------------
  const uint32_t* cab = B.cab[cur] + (size_t)e * C;
  const float2* cimp = B.cimp[cur] + (size_t)e * C;
  const int step_count = B.step_count[e];
  const int M = B.ccount[cur][e];
  float2 p[BPT], v[BPT], tg[BPT];
  float ang[BPT], slp[BPT];
  float4 fo[BPT];
  int a0[BPT], a1[BPT], a2[BPT];
  float ax[BPT], ay[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    p[j] = v[j] = tg[j] = make_float2(0.0f, 0.0f);
    ang[j] = slp[j] = 0.0f;
    fo[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    a0[j] = a1[j] = a2[j] = 1;
    ax[j] = ay[j] = 0.0f;
    if (i < N) {
      p[j] = B.pos[ag[j]];
      v[j] = B.vel[ag[j]];
      ang[j] = B.angle[ag[j]];
      fo[j] = B.fat[ag[j]];
      slp[j] = B.sleep[ag[j]];
      if constexpr (!kT) {
        if (P.action_mode == MACM_ACTION_DISCRETE) {
          const uint8_t* a = (const uint8_t*)actions + ag[j] * 3;
          a0[j] = a[0]; a1[j] = a[1]; a2[j] = a[2];
        } else {
          const float2 c = ((const float2*)actions)[ag[j]];
          ax[j] = c.x; ay[j] = c.y;
        }
        tg[j] = B.targets[(size_t)e * P.n_targets + B.tidx[i]];
      }
      s_c[i] = p[j];  // TDM: dead bodies' positions too (the observation)
    }
  }
  for (int q = tid; q < (N + 31) / 32; q += BS) s_oldc[q] = 0u;
  for (int q = tid; q < N + 2; q += BS) s_deg[q] = 0u;
  if (tid < 7) s_misc[tid] = 0;  // [7]: the slot (acquire_slot)

  // ---- actions -> angle, force (mvmnt.py:97-129) -------------------------------------------
  float Fx[BPT], Fy[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    Fx[j] = Fy[j] = 0.0f;
    if constexpr (kT) {
      if (act[j]) {
        Fx[j] = F[j].x;  // already m_force = 0 + F (the TDM step's action loop)
        Fy[j] = F[j].y;
      }
    } else if (act[j]) {
      if (P.action_mode == MACM_ACTION_DISCRETE) {
        float af = (float)((double)ang[j] + ((double)(a2[j] - 1) * P.rot_step) * P.inv_hz);
        const double ad = (double)af;
        if (fabs(ad) > M_PI) af = (float)(ad - sgn(ad) * (2.0 * M_PI));
        ang[j] = af;
        const double cc = ((a0[j] != 1) && (a1[j] != 1)) ? P.diag_c : 1.0;
        const double k0 = (double)(a0[j] - 1), k1 = (double)(a1[j] - 1);
        double s0, c0, s1, c1;
        act_trig(af, &s0, &c0, &s1, &c1);
        Fx[j] = (float)((c0 * k0 + c1 * k1) * cc * P.force);
        Fy[j] = (float)((s0 * k0 + s1 * k1) * cc * P.force);
      } else {
        float x = ax[j], y = ay[j];
        if ((x * x + y * y) > 1.0f) {  // mvmnt.py:124-126 (the updated x, signs dropped)
          x = sqrtf(x * x / (x * x + y * y));
          y = sqrtf(y * y / (x * x + y * y));
        }
        Fx[j] = x * P.force_f32;
        Fy[j] = y * P.force_f32;
      }
      Fx[j] = 0.0f + Fx[j];  // m_force += force, from ClearForces' zero
      Fy[j] = 0.0f + Fy[j];
    }
  }
  __syncthreads();

  SSTAMP(1);
  // ---- Collide: ordered compaction of the touching contacts (list order) ----------------------
  const float rr = (P.radius + P.radius) * (P.radius + P.radius);
  const float dt_ratio = step_count > 0 ? P.inv_dt * P.dt : 0.0f;  // m_inv_dt0 * dt
  int T = 0;
  for (int k0 = 0; k0 < M; k0 += BS) {
    const int k = k0 + tid;
    bool touch = false;
    uint32_t ab = 0u;
    float2 lam = make_float2(0.0f, 0.0f);
    if (k < M) {
      ab = cab[k];
      lam = cimp[k];
      const int a = ab & 0xffffu, b = ab >> 16;
      // TDM: the contacts of a dead body were destroyed with its proxy (combat.py:162)
      if (live2(a, b)) {
        const float2 pa = s_c[a], pb = s_c[b];
        const float dx = pb.x - pa.x, dy = pb.y - pa.y;
        touch = !(dx * dx + dy * dy > rr);  // b2CollideCircles
        atomicOr(&s_oldc[a >> 5], 1u << (a & 31));
        atomicOr(&s_oldc[b >> 5], 1u << (b & 31));
      }
    }
    int pos;
    const int n = block_scan_excl(touch ? 1 : 0, pos, s_scan);
    if (touch) {
      g_tab[T + pos] = ab;
      g_lam[T + pos] = P.warm_starting ? make_float2(dt_ratio * lam.x, dt_ratio * lam.y) : make_float2(0.0f, 0.0f);
    }
    T += n;
  }
  __syncthreads();

  SSTAMP(2);
  // ---- CSR touching edges, each body's segment in list (= Box2D edge) order -------------------
  for (int t = tid; t < T; t += BS) {
    const uint32_t ab = g_tab[t];
    atomicAdd(&s_deg[ab & 0xffffu], 1u);
    atomicAdd(&s_deg[ab >> 16], 1u);
  }
  __syncthreads();
  int deg[BPT];
  {
    int base = 0;  // the offsets of the chunks before (body order)
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int i = tid + j * BS;
      deg[j] = act[j] ? (int)s_deg[i] : 0;
      int off;
      const int tot = block_scan_excl(deg[j], off, s_scan);
      if (i < N) s_off[i] = (uint32_t)(base + off);  // TDM: dead bodies too (s_off[b + 1] ends body b's edges)
      const unsigned long long m = __ballot(act[j] && deg[j] > 0);  // DFS seeds / unvisited bodies
      if ((tid & (W - 1)) == 0 && i / W < (N + 63) / 64) s_todo[i / W] = m;
      base += tot;
    }
    if (tid == 0) s_off[N] = (uint32_t)(2 * T);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < BPT; ++j)
    if (act[j]) s_deg[tid + j * BS] = s_off[tid + j * BS];  // fill cursor
  __syncthreads();
  for (int t = tid; t < T; t += BS) {
    const uint32_t ab = g_tab[t];
    g_adj[atomicAdd(&s_deg[ab & 0xffffu], 1u)] = (uint32_t)t;
    g_adj[atomicAdd(&s_deg[ab >> 16], 1u)] = (uint32_t)t;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    if (act[j] && deg[j] > 1) {  // insertion sort back into list order == Box2D edge order
      const int o0 = (int)s_off[tid + j * BS];
      for (int x = o0 + 1; x < o0 + deg[j]; ++x) {
        const uint32_t key = g_adj[x];
        int y = x - 1;
        while (y >= o0 && g_adj[y] > key) {
          g_adj[y + 1] = g_adj[y];
          --y;
        }
        g_adj[y + 1] = key;
      }
    }
  }
  __syncthreads();

  SSTAMP(3);
  // ---- island DFS in Box2D order, serial on thread 0 ---------------------------------------------
  // Seeds: bodies with touching edges, highest index first (reverse creation order). A body is
  // visited once its s_todo bit is cleared; a contact once bit 31 of its g_tab entry is set
  // (b < 32768). One thread does every global access of the walk, so program order orders them.
  if (tid == 0) {
    int nord = 0, nisl = 0, nb = 0;
    for (int w = (N + 63) / 64 - 1; w >= 0;) {
      const unsigned long long m = s_todo[w];
      if (m == 0ull) {
        --w;
        continue;
      }
      const int s = w * 64 + 63 - __clzll(m);
      s_todo[w] = m & ~(1ull << (s & 63));
      s_ic[nisl] = (uint32_t)nord;
      s_ib[nisl] = (uint16_t)nb;
      int sp = 0;
      s_stk[sp++] = (uint16_t)s;
      while (sp > 0) {
        const int b = s_stk[--sp];
        s_ibod[nb++] = (uint16_t)b;
        const int e0 = (int)s_off[b], e1 = (int)s_off[b + 1];
        for (int q = e0; q < e1; ++q) {
          const int t = (int)g_adj[q];
          const uint32_t ab = g_tab[t];
          if (ab & 0x80000000u) continue;
          g_tab[t] = ab | 0x80000000u;
          g_ord[nord++] = (uint32_t)t;
          const int a = ab & 0xffffu, bb = ab >> 16;
          const int o = (a == b) ? bb : a;
          const unsigned long long ob = 1ull << (o & 63);
          const unsigned long long tw = s_todo[o >> 6];
          if (!(tw & ob)) continue;
          s_todo[o >> 6] = tw & ~ob;
          s_stk[sp++] = (uint16_t)o;
        }
      }
      ++nisl;
    }
    s_ic[nisl] = (uint32_t)nord;
    s_ib[nisl] = (uint16_t)nb;
    s_misc[0] = nisl;
  }
  __syncthreads();
  const int nisl = s_misc[0];
  const int nord = nisl > 0 ? (int)s_ic[nisl] : 0;

  SSTAMP(4);
  // ---- integrate velocities + damping; island-ordered records with normals --------------------
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    if (act[j]) {
      const float vx = v[j].x + P.dt * (0.0f + P.inv_mass * Fx[j]);  // gravityScale * gravity == 0
      const float vy = v[j].y + P.dt * (0.0f + P.inv_mass * Fy[j]);
      s_v[tid + j * BS] = make_float2(vx * P.damp, vy * P.damp);
    }
  }
  for (int k = tid; k < nord; k += BS) {
    const int t = (int)g_ord[k];
    const uint32_t ab = g_tab[t] & 0x7fffffffu;
    const int a = ab & 0xffffu, b = ab >> 16;
    const float2 pa = s_c[a], pb = s_c[b];
    float nx = 1.0f, ny = 0.0f;  // InitializeVelocityConstraints: (1, 0) when the centres coincide
    const float ddx = pa.x - pb.x, ddy = pa.y - pb.y;
    if (ddx * ddx + ddy * ddy > kEps * kEps) {
      nx = pb.x - pa.x;
      ny = pb.y - pa.y;
      normalize(nx, ny);
    }
    g_cst[k] = make_float4(__uint_as_float(ab), nx, ny, 0.0f);
    g_cim[k] = g_lam[t];
  }
  __syncthreads();

  const float mA = P.inv_mass, mB = P.inv_mass;
  const float kmass = (mA + mB) > 0.0f ? 1.0f / (mA + mB) : 0.0f;  // normalMass == tangentMass
  const float friction = P.friction;

  // ---- LEVELS (the workgroup callers: worlds above 1024 agents, TDM above 64, dense workgroup envs):
  //      Gauss-Seidel levels, as the workgroup path's kernel B --------------------------------------
  // level(k) = 1 + the level of the last earlier contact (island order) sharing a body with k, so a
  // level's contacts share no body and every body keeps Box2D's sequence of updates; one wave then
  // steps the levels with 64 contacts at a time instead of one thread per island walking its
  // contacts one by one (round 5). The records stay in island order (g_cst, g_cim); g_lidx lists
  // them in level order. Working arrays dead by now: g_adj (the walk's CSR edges), g_tab (the
  // touching pairs, read by the records above), s_deg, s_off, s_stk, s_slp.
  uint32_t* g_lvl = g_adj;       // [nord] level | island << 16 of island-order contact k
  uint32_t* g_lidx = g_adj + C;  // [nord] the island-order index of the p-th contact in level order
  uint32_t* g_hist = g_tab;      // [levels] counts, then positions
  auto level_body = [&](float4 r, float2& im, bool warm, float2& va, float2& vb) {
    // the contact update on (x, y) pairs (v_pk_mul / v_pk_add): the same IEEE operations as the
    // scalar form, contraction off
    const float nx = r.y, ny = r.z;
    const lpf2 n = {nx, ny}, t = {ny, -nx};
    lpf2 vA = {va.x, va.y}, vB = {vb.x, vb.y};
    if (warm) {
      const lpf2 Pv = im.x * n + im.y * t;
      vA = vA - mA * Pv;
      vB = vB + mB * Pv;
    } else {
      {
        const lpf2 pr = (vB - vA) * t;
        float lambda = kmass * (-(pr.x + pr.y));
        const float maxf = friction * im.x;
        const float ni = sclamp(im.y + lambda, -maxf, maxf);
        lambda = ni - im.y;
        im.y = ni;
        const lpf2 Pv = lambda * t;
        vA = vA - mA * Pv;
        vB = vB + mB * Pv;
      }
      {
        const lpf2 pr = (vB - vA) * n;
        float lambda = -kmass * ((pr.x + pr.y) - 0.0f);
        const float ni = fmaxf(im.x + lambda, 0.0f);
        lambda = ni - im.x;
        im.x = ni;
        const lpf2 Pv = lambda * n;
        vA = vA - mA * Pv;
        vB = vB + mB * Pv;
      }
    }
    va = make_float2(vA.x, vA.y);
    vb = make_float2(vB.x, vB.y);
  };
  // one wave walks the level-ordered contacts in chunks of 64 (one per lane, loaded a chunk ahead); in
  // a chunk it steps its levels, the lanes of the current level updating together and the others on a
  // dummy LDS slot (branch-free); a level cut by a chunk boundary is finished in the next chunk
  struct LSlot {
    float4 r;
    float2 m;
    uint32_t li;
    int k;
  };
  const int nlev_chunks = (nord + W - 1) / W;
  auto lload = [&](int c, LSlot& x) {
    const int q = min(c * W + (tid & (W - 1)), nord - 1);
    x.k = (int)g_lidx[q];
    x.r = g_cst[x.k];
    x.m = g_cim[x.k];
    x.li = g_lvl[x.k];
  };
  auto lwait = [&]() { __builtin_amdgcn_s_waitcnt(0x0f70); };  // vmcnt(0)
  auto lsync = [&]() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); };
  auto lchunk = [&](int c, const LSlot& x, int& rel, int& nsteps) {
    const int lane = tid & (W - 1);
    const bool valid = c * W + lane < nord;
    const int mylv = valid ? (int)(x.li & 0xffffu) : 0x7fff;
    const int lv0 = __builtin_amdgcn_readfirstlane(mylv);
    const int lv1 = __builtin_amdgcn_readlane(mylv, min(W, nord - c * W) - 1);
    rel = valid ? mylv - lv0 : 0x7fff;
    nsteps = lv1 - lv0 + 1;
  };
  bool leveled = false;
  // few touching contacts (sparse envs): the islands' own threads are as fast and skip the set-up
  // (TDM 2 x 64 at 1024 envs: +2% with levels; 2 x 256: -38%)
  constexpr int kLevelMinContacts = 64;
  if (LEVELS && nord >= kLevelMinContacts) {
    for (int q = tid; q < N + 2; q += BS) s_deg[q] = 0u;
    __syncthreads();
    if (tid == 0) {  // the levels, serial in island order (its pairs read 16 records ahead)
      int dmax = 0, I = 0;
      constexpr int LA = 16;
      uint32_t abq[LA];
#pragma unroll
      for (int j = 0; j < LA; ++j) abq[j] = __float_as_uint(g_cst[min(j, max(nord - 1, 0))].x);
      for (int k0 = 0; k0 < nord; k0 += LA) {
#pragma unroll
        for (int j = 0; j < LA; ++j) {
          const int k = k0 + j;
          if (k >= nord) continue;
          const uint32_t ab = abq[j];
          abq[j] = __float_as_uint(g_cst[min(k + LA, nord - 1)].x);
          while (I + 1 < nisl && (int)s_ic[I + 1] <= k) ++I;
          const int a = ab & 0xffffu, b = ab >> 16;
          const int l = (int)max(s_deg[a], s_deg[b]);
          s_deg[a] = s_deg[b] = (uint32_t)(l + 1);
          g_lvl[k] = (uint32_t)l | ((uint32_t)I << 16);
          dmax = max(dmax, l + 1);
        }
      }
      s_misc[2] = dmax;
    }
    __syncthreads();
    const int nlev = s_misc[2];
    for (int q = tid; q < nlev; q += BS) g_hist[q] = 0u;
    __syncthreads();
    for (int k = tid; k < nord; k += BS) atomicAdd(&g_hist[g_lvl[k] & 0xffffu], 1u);
    __syncthreads();
    {  // exclusive scan of the level counts
      int base = 0;
      for (int q0 = 0; q0 < nlev; q0 += BS) {
        const int q = q0 + tid;
        const int c = q < nlev ? (int)g_hist[q] : 0;
        int off;
        const int tot = block_scan_excl(c, off, s_scan);
        if (q < nlev) g_hist[q] = (uint32_t)(base + off);
        base += tot;
        __syncthreads();
      }
    }
    __syncthreads();
    for (int k = tid; k < nord; k += BS) g_lidx[atomicAdd(&g_hist[g_lvl[k] & 0xffffu], 1u)] = (uint32_t)k;
    __syncthreads();
    leveled = true;
    if (tid < W && nord > 0) {
      float2* const s_dum = reinterpret_cast<float2*>(s_off);  // the walk's CSR offsets: dead
      auto vel_pass = [&](bool warm) {
        LSlot cur, nxt;
        lload(0, cur);
        lwait();
        for (int c = 0; c < nlev_chunks; ++c) {
          lload(c + 1, nxt);
          int rel, nsteps;
          lchunk(c, cur, rel, nsteps);
          const uint32_t ab = __float_as_uint(cur.r.x);
          float2* const pa0 = s_v + (ab & 0xffffu);
          float2* const pb0 = s_v + (ab >> 16);
          float2* const pd = s_dum;  // one shared dummy slot
          float2 im = cur.m;
          for (int i = 0; i < nsteps; ++i) {
            const bool on = rel == i;
            float2* const pa = on ? pa0 : pd;
            float2* const pb = on ? pb0 : pd;
            float2 va = *pa, vb = *pb;
            float2 lm = im;
            level_body(cur.r, lm, warm, va, vb);
            *pa = va;
            *pb = vb;
            im = on ? lm : im;
            lsync();
          }
          if (!warm && c * W + (tid & (W - 1)) < nord) g_cim[cur.k] = im;
          lwait();
          cur = nxt;
        }
      };
      if (P.warm_starting) vel_pass(true);
      for (int it = 0; it < P.vel_iters; ++it) vel_pass(false);
    }
  }

  SSTAMP(5);
  // ---- warm start + velocity iterations, one thread per island (b2ContactSolver) ---------------
  // The records are in HBM (the slot's arrays): an island's thread reads them kSpillChunk at a time,
  // all loads of a chunk issued before its first update (round 5: one L2 round trip per chunk on the
  // serial chain instead of one per contact; the updates themselves are unchanged and in order)
  // (the wave kernels' dense-env fallback, RECS_LDS, keeps one record at a time: its registers are the
  // wave kernel's, whose occupancy a larger chunk would cost)
  constexpr int U = RECS_LDS ? 1 : (BPT >= 4 ? kSpillChunk / 2 : kSpillChunk);
  for (int I = leveled ? nisl : tid; I < nisl; I += BS) {
    const int c0 = (int)s_ic[I], c1 = (int)s_ic[I + 1];
    auto chunk = [&](int k0, float4* r, float2* im) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int k = min(k0 + j, c1 - 1);
        r[j] = g_cst[k];
        im[j] = g_cim[k];
      }
    };
    if (P.warm_starting) {
      for (int k0 = c0; k0 < c1; k0 += U) {
        float4 r[U];
        float2 im[U];
        chunk(k0, r, im);
#pragma unroll
        for (int j = 0; j < U; ++j) {
          if (k0 + j >= c1) break;
          const uint32_t ab = __float_as_uint(r[j].x);
          const int a = ab & 0xffffu, b = ab >> 16;
          const float nx = r[j].y, ny = r[j].z, tx = ny, ty = -nx;  // b2Cross(normal, 1.0f)
          const float Px = im[j].x * nx + im[j].y * tx, Py = im[j].x * ny + im[j].y * ty;
          float2 va = s_v[a], vb = s_v[b];
          va.x = va.x - mA * Px;
          va.y = va.y - mA * Py;
          vb.x = vb.x + mB * Px;
          vb.y = vb.y + mB * Py;
          s_v[a] = va;
          s_v[b] = vb;
        }
      }
    }
    for (int it = 0; it < P.vel_iters; ++it) {
      for (int k0 = c0; k0 < c1; k0 += U) {
        float4 r[U];
        float2 imc[U];
        chunk(k0, r, imc);
#pragma unroll
        for (int j = 0; j < U; ++j) {
          if (k0 + j >= c1) break;
          float2 im = imc[j];
          const uint32_t ab = __float_as_uint(r[j].x);
          const int a = ab & 0xffffu, b = ab >> 16;
          const float nx = r[j].y, ny = r[j].z, tx = ny, ty = -nx;
          float2 va = s_v[a], vb = s_v[b];
          {  // tangent first
            const float dvx = vb.x - va.x, dvy = vb.y - va.y;
            const float vt = dvx * tx + dvy * ty;
            float lambda = kmass * (-vt);
            const float maxf = friction * im.x;
            const float ni = sclamp(im.y + lambda, -maxf, maxf);
            lambda = ni - im.y;
            im.y = ni;
            const float Px = lambda * tx, Py = lambda * ty;
            va.x = va.x - mA * Px; va.y = va.y - mA * Py;
            vb.x = vb.x + mB * Px; vb.y = vb.y + mB * Py;
          }
          {  // normal (velocityBias == 0: restitution 0)
            const float dvx = vb.x - va.x, dvy = vb.y - va.y;
            const float vn = dvx * nx + dvy * ny;
            float lambda = -kmass * (vn - 0.0f);
            const float ni = fmaxf(im.x + lambda, 0.0f);
            lambda = ni - im.x;
            im.x = ni;
            const float Px = lambda * nx, Py = lambda * ny;
            va.x = va.x - mA * Px; va.y = va.y - mA * Py;
            vb.x = vb.x + mB * Px; vb.y = vb.y + mB * Py;
          }
          s_v[a] = va;
          s_v[b] = vb;
          g_cim[k0 + j] = im;
        }
      }
    }
  }
  __syncthreads();
  for (int k = tid; k < nord; k += BS) g_lam[g_ord[k]] = g_cim[k];  // StoreImpulses, list order

  SSTAMP(6);
  // ---- integrate positions ----------------------------------------------------------------------
  float cx[BPT], cy[BPT], vx[BPT], vy[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    cx[j] = p[j].x;
    cy[j] = p[j].y;
    vx[j] = vy[j] = 0.0f;
    if (act[j]) {
      const float2 vv = s_v[tid + j * BS];
      vx[j] = vv.x;
      vy[j] = vv.y;
      const float tx = P.dt * vx[j], ty = P.dt * vy[j];
      if (tx * tx + ty * ty > kMaxTranslation * kMaxTranslation) {
        const float ratio = kMaxTranslation / sqrtf(tx * tx + ty * ty);
        vx[j] = vx[j] * ratio;
        vy[j] = vy[j] * ratio;
      }
      cx[j] = cx[j] + P.dt * vx[j];
      cy[j] = cy[j] + P.dt * vy[j];
      s_c[tid + j * BS] = make_float2(cx[j], cy[j]);
    }
  }
  __syncthreads();

  SSTAMP(7);
  if (leveled) {
    // the position passes by levels (LEVELS), as kernel B: an island leaves after the
    // first pass whose minimum separation (from 0) is >= -3 linearSlop; the minimum by LDS float
    // atomics (order-independent), the islands' flags in s_isolv
    for (int I = tid; I < nisl; I += BS) s_isolv[I] = 0;
    __syncthreads();
    if (tid < W && nord > 0) {
      float* const s_mins = s_slp;                              // [nisl] (the sleep clocks come later)
      float2* const pdd = reinterpret_cast<float2*>(s_off);     // a shared dummy slot
      float* const pmd = reinterpret_cast<float*>(s_off) + 2 + (tid & (W - 1));  // a dummy minimum per lane
      const float K = mA + mB;
      for (int it = 0; it < P.pos_iters; ++it) {
        for (int I = tid; I < nisl; I += W) s_mins[I] = 0.0f;
        lsync();
        LSlot cur, nxt;
        lload(0, cur);
        lwait();
        for (int c = 0; c < nlev_chunks; ++c) {
          lload(c + 1, nxt);
          int rel, nsteps;
          lchunk(c, cur, rel, nsteps);
          const int I = (int)(cur.li >> 16);
          const bool live = c * W + (tid & (W - 1)) < nord && !s_isolv[I];
          const int relp = live ? rel : 0x7fff;
          const uint32_t ab = __float_as_uint(cur.r.x);
          float2* const pca = s_c + (ab & 0xffffu);
          float2* const pcb = s_c + (ab >> 16);
          for (int i = 0; i < nsteps; ++i) {
            const bool on = relp == i;
            float2* const pa = on ? pca : pdd;
            float2* const pb = on ? pcb : pdd;
            float* const pm = on ? s_mins + I : pmd;
            const float2 ca = *pa, cb = *pb;
            const lpf2 cA = {ca.x, ca.y}, cB = {cb.x, cb.y};
            const lpf2 d = cB - cA, d2 = d * d;
            const float len = sqrt_rn(d2.x + d2.y);
            const lpf2 n = len < kEps ? d : d * rcp_rn(len);  // b2Vec2::Normalize
            const lpf2 pr = d * n;
            const float sep = (pr.x + pr.y) - P.radius - P.radius;
            const float Cc = sclamp(kBaumgarte * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
            const float imp = K > 0.0f ? div_by_invariant(-Cc, K) : 0.0f;
            const lpf2 Pv = imp * n, nA = cA - mA * Pv, nB = cB + mB * Pv;
            *pa = make_float2(nA.x, nA.y);
            *pb = make_float2(nB.x, nB.y);
            __hip_atomic_fetch_min(pm, sep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            lsync();
          }
          lwait();
          cur = nxt;
        }
        lsync();
        bool open = false;
        for (int I = tid; I < nisl; I += W) {
          if (s_isolv[I]) continue;
          if (s_mins[I] >= -3.0f * kLinearSlop) s_isolv[I] = 1;
          else open = true;
        }
        lsync();
        if (__ballot(open) == 0ull) break;
      }
    }
    __syncthreads();
  }
  // ---- position iterations, one thread per island (early exit at -3 linearSlop) ---------------------
  for (int I = leveled ? nisl : tid; I < nisl; I += BS) {
    const int c0 = (int)s_ic[I], c1 = (int)s_ic[I + 1];
    int solved = 0;
    for (int it = 0; it < P.pos_iters; ++it) {
      float min_sep = 0.0f;
      for (int k0 = c0; k0 < c1; k0 += U) {
        uint32_t abc[U];  // the chunk's pairs, loaded before its first update
#pragma unroll
        for (int j = 0; j < U; ++j) abc[j] = __float_as_uint(g_cst[min(k0 + j, c1 - 1)].x);
#pragma unroll
        for (int j = 0; j < U; ++j) {
        if (k0 + j >= c1) break;
        const uint32_t ab = abc[j];
        const int a = ab & 0xffffu, b = ab >> 16;
        float2 ca = s_c[a], cb = s_c[b];
        float nx = cb.x - ca.x, ny = cb.y - ca.y;
        normalize(nx, ny);
        const float sep = ((cb.x - ca.x) * nx + (cb.y - ca.y) * ny) - P.radius - P.radius;
        min_sep = bmin(min_sep, sep);
        const float Cc = sclamp(kBaumgarte * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
        const float K = mA + mB;
        const float imp = K > 0.0f ? div_by_invariant(-Cc, K) : 0.0f;
        const float Px = imp * nx, Py = imp * ny;
        ca.x = ca.x - mA * Px; ca.y = ca.y - mA * Py;
        cb.x = cb.x + mB * Px; cb.y = cb.y + mB * Py;
        s_c[a] = ca;
        s_c[b] = cb;
        }
      }
      if (min_sep >= -3.0f * kLinearSlop) {
        solved = 1;
        break;
      }
    }
    s_isolv[I] = (uint8_t)solved;
  }

  SSTAMP(8);
  // ---- sleep clock + island sleep decision (b2Island::Solve) --------------------------------------
  float ns[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    ns[j] = 0.0f;
    if (act[j]) {
      const bool moving = vx[j] * vx[j] + vy[j] * vy[j] > kLinearSleepTol * kLinearSleepTol;
      ns[j] = moving ? 0.0f : slp[j] + P.dt;
      s_slp[tid + j * BS] = ns[j];
      s_flag[tid + j * BS] = (deg[j] == 0 && ns[j] >= kTimeToSleep && P.pos_iters > 0) ? 1 : 0;
    }
  }
  __syncthreads();
  for (int I = tid; I < nisl; I += BS) {
    const int b0 = s_ib[I], b1 = s_ib[I + 1];
    float mn = 3.402823466e+38f;
    for (int k = b0; k < b1; ++k) mn = bmin(mn, s_slp[s_ibod[k]]);
    const uint8_t sl = (mn >= kTimeToSleep && s_isolv[I]) ? 1 : 0;
    for (int k = b0; k < b1; ++k) s_flag[s_ibod[k]] = sl;
  }
  __syncthreads();

  // ---- SynchronizeFixtures: fat-AABB hysteresis ------------------------------------------------------
  float4 fn[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    fn[j] = fo[j];
    if (act[j]) {
      const float2 cc = s_c[i];
      cx[j] = cc.x;
      cy[j] = cc.y;
      const float r = P.radius;
      const float c0x = p[j].x, c0y = p[j].y;
      const float lox = bmin(c0x - r, cx[j] - r), loy = bmin(c0y - r, cy[j] - r);
      const float hix = bmax(c0x + r, cx[j] + r), hiy = bmax(c0y + r, cy[j] + r);
      const bool contains = fo[j].x <= lox && fo[j].y <= loy && hix <= fo[j].z && hiy <= fo[j].w;
      if (!contains) {
        fn[j] = make_float4(lox - kAabbExtension, loy - kAabbExtension, hix + kAabbExtension, hiy + kAabbExtension);
        const float dx = kAabbMultiplier * (cx[j] - c0x), dy = kAabbMultiplier * (cy[j] - c0y);
        if (dx < 0.0f) fn[j].x += dx; else fn[j].z += dx;
        if (dy < 0.0f) fn[j].y += dy; else fn[j].w += dy;
      }
      if (s_flag[i]) {
        vx[j] = 0.0f;
        vy[j] = 0.0f;
        ns[j] = 0.0f;
      }
      Rec r0;
      r0.fn = fn[j];
      r0.fo = fo[j];
      r0.c = make_float2(cx[j], cy[j]);
      recs[i] = r0;
    } else if (kT && i < N) {  // a dead body: overlaps nothing, infinitely far
      Rec r0;
      r0.fn = r0.fo = make_float4(__builtin_inff(), __builtin_inff(), -__builtin_inff(), -__builtin_inff());
      r0.c = make_float2(__builtin_inff(), __builtin_inff());
      recs[i] = r0;
    }
  }
  __syncthreads();

  SSTAMP(9);
  // ---- all-pairs sweep: collisions, new-pair counts, nearest neighbour (mvmnt.py:185-196) ------------
  //   world.contacts after the step = Ov(F_{t-1}) U Ov(F_t); new contacts = Ov(F_t) \ Ov(F_{t-1})
  bool coll[BPT];
  int newcnt[BPT], bj[BPT];
  float best[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    coll[j] = act[j] && ((s_oldc[i >> 5] >> (i & 31)) & 1u);
    newcnt[j] = 0;
    best[j] = __builtin_inff();
    bj[j] = i == 0 ? 1 : 0;
    if (act[j]) {
      for (int q = 0; q < N; ++q) {
        const Rec r = recs[q];
        const bool ovn = overlap(fn[j], r.fn);
        const float dx = r.c.x - cx[j], dy = r.c.y - cy[j];
        const float d2 = dx * dx + dy * dy;  // b2DistanceSquared(other, agent)
        const bool other = q != i;
        coll[j] |= other && ovn;
        if (other && d2 < best[j]) {  // strict '<': the lowest index wins ties (mvmnt.py:194)
          best[j] = d2;
          bj[j] = q;
        }
        if (q > i && ovn && !overlap(fo[j], r.fo)) ++newcnt[j];
      }
    }
  }
  SSTAMP(10);
  // ---- next ordered list: new pairs (a desc, b desc) ++ surviving old pairs -------------------------
  uint32_t* ocab = B.cab[nxt] + (size_t)e * C;
  float2* ocimp = B.cimp[nxt] + (size_t)e * C;
  int excl[BPT];
  int nnew = 0;  // the chunks' exclusive scans in body order, then the total
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int tot = block_scan_excl(newcnt[j], excl[j], s_scan);
    excl[j] += nnew;
    nnew += tot;
  }
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int i = tid + j * BS;
    if (act[j] && newcnt[j] > 0) {
      int w = nnew - excl[j] - newcnt[j];  // agents > i come first
      for (int q = N - 1; q > i; --q) {
        const Rec r = recs[q];
        if (overlap(fn[j], r.fn) && !overlap(fo[j], r.fo)) {
          if (w < C) {
            ocab[w] = (uint32_t)i | ((uint32_t)q << 16);
            ocimp[w] = make_float2(0.0f, 0.0f);
          }
          ++w;
        }
      }
    }
  }
  int kept = 0, Tr = 0;
  for (int k0 = 0; k0 < M; k0 += BS) {
    const int k = k0 + tid;
    bool keep = false, touch = false;
    uint32_t ab = 0u;
    if (k < M) {
      ab = cab[k];
      const int a = ab & 0xffffu, b = ab >> 16;
      keep = overlap(recs[a].fn, recs[b].fn);
      // touching at Collide, from the start-of-step positions (the state is not yet written back)
      const float2 pa = B.pos[(size_t)e * N + a], pb = B.pos[(size_t)e * N + b];
      const float dx = pb.x - pa.x, dy = pb.y - pa.y;
      touch = !(dx * dx + dy * dy > rr) && live2(a, b);
    }
    int tpos, kpos;
    const int tn = block_scan_excl(touch ? 1 : 0, tpos, s_scan);
    const int kn = block_scan_excl(keep ? 1 : 0, kpos, s_scan);
    if (keep) {
      const int w = nnew + kept + kpos;
      if (w < C) {
        ocab[w] = ab;
        ocimp[w] = touch ? g_lam[Tr + tpos] : make_float2(0.0f, 0.0f);
      }
    }
    Tr += tn;
    kept += kn;
  }
  int status = 0;
  int total = nnew + kept;
  if (total > C) {
    status |= MACM_ST_CONTACT_OVERFLOW;
    total = C;
  }

  // ---- TDM: state write-back, TDM.get_obs (combat.py:166-167, 206-227), done / winner (:171-182) --------
  if constexpr (kT) {
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int i = tid + j * BS;
      if (i < N) {
        if (act[j]) {
          B.pos[ag[j]] = make_float2(cx[j], cy[j]);
          B.vel[ag[j]] = make_float2(vx[j], vy[j]);
          B.fat[ag[j]] = fn[j];
          B.sleep[ag[j]] = ns[j];
        }
        s_slp[i] = ang[j];  // the sleep clocks are dead: the angles for the observation
      }
    }
    // the observation reads only LDS: the slot goes back to the pool before the O(N^2) obs writes
    // (release_slot's barrier also orders the s_slp writes before the obs reads)
    release_slot(B, slot);
    __syncthreads();
    const size_t rows = (size_t)e * N * (N - 1);
    if (TB->snap_out) {  // the split observation (tdm_obs_snap.hip): the pose snapshot instead
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        const int i = tid + j * BS;
        if (i < N) st_wt4(TB->snap_out + (size_t)e * N + i, make_float4(s_c[i].x, s_c[i].y, s_slp[i], act[j] ? 1.0f : 0.0f));
      }
    } else if (wide) {
      tdm_obs_block_linear<OT>(obs ? obs + rows * 4 : nullptr, TB->mask_out ? TB->mask_out + rows : nullptr, N, tid,
                               BS, s_alivew, *TP, s_c, s_slp);
    } else {
      tdm_obs_pairs<OT>(obs ? obs + rows * 4 : nullptr, TB->mask_out ? TB->mask_out + rows : nullptr, N, tid, livem,
                        *TP, s_c, s_slp);
    }
    int alive_teams = 0, last_team = -1;
    for (int t = 0; t < TP->n_teams; ++t) {
      bool any = false;
#pragma unroll
      for (int j = 0; j < BPT; ++j) any |= act[j] && tdm_team_of(*TP, tid + j * BS) == t;
      if (__syncthreads_or(any)) {
        ++alive_teams;
        last_team = t;
      }
    }
    if (tid == 0) {
      const double tp = B.time_passed[e] + P.inv_hz;  // time_passed += 1/hz
      uint8_t dn = tp > P.time_limit ? 1 : 0;
      int win = TB->winner[e];
      if (B.done[e]) dn = 1;  // done latches
      if (alive_teams == 1) {
        dn = 1;
        win = last_team;
      }
      if (alive_teams == 0) dn = 1;
      TB->winner[e] = win;
      if (TB->winner_out) TB->winner_out[e] = win;
      B.time_passed[e] = tp;
      B.done[e] = dn;
      if (done_out) done_out[e] = dn;
      B.step_count[e] = step_count + 1;
      B.ccount[nxt][e] = total;
      if (status) {
        B.status[e] |= status;
        report_status(B, status);
      }
      B.env_counters[(size_t)e * 4 + 3] += (unsigned long long)dn;  // counters 0-2: the wave kernel
      if (B.spill_count) B.spill_count[e] += 1u;
    }
  } else {
    // ---- rewards (mvmnt.py:160-179) + obs (mvmnt.py:181-222) -------------------------------------------
    float rew[BPT];
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      rew[j] = 0.0f;
      if (act[j]) {
        const float tdx = tg[j].x - cx[j], tdy = tg[j].y - cy[j];  // target - agent.body.position
        const float td2 = tdx * tdx + tdy * tdy;
        const double d = sqrt((double)td2);
        if (coll[j]) rew[j] = -1.0f;
        else if (P.reward_mode == MACM_REWARD_LINEAR) rew[j] = (float)((-d / 35) + 1);
        else rew[j] = (d < P.reward_radius) ? 1.0f : 0.0f;
        rew_out[ag[j]] = rew[j];
        if (coll_out) coll_out[ag[j]] = coll[j] ? 1 : 0;
        if (nbr_out) nbr_out[ag[j]] = bj[j];
        if (obs) {
          const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
          const float2 cb = recs[bj[j]].c;
          write_obs<OT>(obs + ag[j] * od, P.coord, ang[j], best[j], cb.x - cx[j], cb.y - cy[j], tdx, tdy, td2);
        }
      }
    }
    int dummy, ncoll = 0, npos = 0;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      ncoll += block_scan_excl(act[j] && coll[j] ? 1 : 0, dummy, s_scan);  // also orders the B.pos reads
      npos += block_scan_excl(act[j] && rew[j] > 0.0f ? 1 : 0, dummy, s_scan);  // before the write-back
    }
    // thread 0: the step's reward sum in agent-slot order (flock_common.hpp); linear rewards only, a
    // binary step sums to npos - ncoll exactly (macm_world_reward_sums)
    double rsum = 0.0;
    const bool lin = P.reward_mode == MACM_REWARD_LINEAR;
    if (lin) {
      if constexpr (BPT == 1) {
        rsum = block_pairwise_sum((double)rew[0], reinterpret_cast<double*>(s_scan));
      } else {
        double* s_grp = reinterpret_cast<double*>(s_slp);  // the sleep clocks are dead: 64-body group sums
        const int gw = BS / W;
#pragma unroll
        for (int j = 0; j < BPT; ++j) {
          const double g = wave_pairwise_sum((double)rew[j]);
          if ((tid & (W - 1)) == 0) s_grp[j * gw + tid / W] = g;
        }
        __syncthreads();
        if (tid == 0) {
          const int ng = BPT * gw;
          int n2 = 1;
          while (n2 < ng) n2 <<= 1;
          for (int q = ng; q < n2; ++q) s_grp[q] = 0.0;
          for (int h = 1; h < n2; h <<= 1)
            for (int q = 0; q + h < n2; q += 2 * h) s_grp[q] = s_grp[q] + s_grp[q + h];
          rsum = s_grp[0];
        }
        __syncthreads();
      }
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      if (act[j]) {
        B.pos[ag[j]] = make_float2(cx[j], cy[j]);
        B.vel[ag[j]] = make_float2(vx[j], vy[j]);
        B.angle[ag[j]] = ang[j];
        B.fat[ag[j]] = fn[j];
        B.sleep[ag[j]] = ns[j];
      }
    }
    if (tid == 0) {
      const double tp = B.time_passed[e] + P.inv_hz;  // time_passed += 1/hz (mvmnt.py:134-136)
      const uint8_t dn = tp > P.time_limit ? 1 : 0;
      B.time_passed[e] = tp;
      B.done[e] = dn;
      if (done_out) done_out[e] = dn;
      B.step_count[e] = step_count + 1;
      B.ccount[nxt][e] = total;
      if (status) {
        B.status[e] |= status;
        report_status(B, status);
      }
      unsigned long long* ec = B.env_counters + (size_t)e * 4;
      ec[0] += (unsigned long long)N;
      ec[1] += (unsigned long long)ncoll;
      ec[2] += (unsigned long long)npos;
      ec[3] += (unsigned long long)dn;
      if (lin) add_reward_sum(B, e, rsum);
      if (B.spill_count) B.spill_count[e] += 1u;
    }
    SSTAMP(11);
    release_slot(B, slot);  // the observation above reads recs (HBM when !RECS_LDS)
  }
}

}  // namespace spill
}  // namespace macm
