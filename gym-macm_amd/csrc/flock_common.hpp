// flock_common.hpp — shared device/host definitions for the batched Flock stepper.
//
// Arithmetic contract: every float expression that mirrors Box2D keeps Box2D's
// operand order and is compiled with -ffp-contract=off, so each op rounds exactly
// as Box2D's SSE2 (no-FMA) build does. Double expressions mirror the reference's
// numpy/Python double math (gym_macm/envs/mvmnt.py) in the same order.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/macm.h"
#include "macm_math.h"

namespace macm {

// Box2D 2.3 b2Settings.h constants used on the path.
constexpr float kEps = 1.1920928955078125e-07f;  // FLT_EPSILON
constexpr float kLinearSlop = 0.005f;
constexpr float kAabbExtension = 0.1f;
constexpr float kAabbMultiplier = 2.0f;
constexpr float kMaxTranslation = 2.0f;
constexpr float kBaumgarte = 0.2f;
constexpr float kMaxLinearCorrection = 0.2f;
constexpr float kTimeToSleep = 0.5f;
constexpr float kLinearSleepTol = 0.01f;
constexpr float kPi32 = 3.14159265359f;  // b2_pi

// Per-launch parameters derived on the host from macm_config exactly as the
// reference derives them (Python double arithmetic / SWIG float conversion).
struct StepParams {
  int32_t n_envs, n_agents, n_targets, max_contacts;  // TDM: n_targets = 0
  int32_t vel_iters, pos_iters, warm_starting;
  int32_t action_mode, reward_mode, coord;
  int32_t force_spill;  // test hook (macm_world_set_debug): every env takes the spill step
  int32_t sweep;        // workgroup pair sweep: 0 = by N (strip cells at N >= 512), 1 = cells, 2 = all pairs
  float dt;          // fl32(1.0 / hz)                       cm_framework.py:182-185 -> world.Step
  float inv_dt;      // 1.0f / dt                            b2World::Step
  float inv_mass;    // 1 / (density * b2_pi * r * r)        b2CircleShape::ComputeMass
  float damp;        // 1 / (1 + dt * linearDamping)         b2Island::Solve
  float radius;      // circle radius
  float friction;    // b2MixFriction = sqrtf(f * f)
  float force_f32;   // (float)agent_force (continuous mode: numpy float32 * int)
  double rot_step;   // rotation_speed, multiplied as ((a2-1) * rot) * (1/hz)   mvmnt.py:103-104
  double inv_hz;     // 1 / hz (Python float division)                       mvmnt.py:104,134
  double force;      // agent_force (double)                                 mvmnt.py:113-116
  double diag_c;     // 1 / np.sqrt(2)                                       mvmnt.py:112
  double reward_radius;
  double time_limit;
};

struct WorldBuffers {
  float2* pos;         // [E, N]
  float2* vel;         // [E, N]
  float* angle;        // [E, N]
  float4* fat;         // [E, N]   (lo.x, lo.y, hi.x, hi.y)
  float* sleep;        // [E, N]
  float2* targets;     // [E, T]
  int32_t* tidx;       // [N]
  int32_t* ccount[2];  // [E]      double-buffered ordered contact list
  uint32_t* cab[2];    // [E, C]   a | b << 16
  float2* cimp[2];     // [E, C]   (normalImpulse, tangentImpulse)
  int32_t* step_count; // [E]
  double* time_passed; // [E]
  uint8_t* done;       // [E]
  int32_t* status;     // [E]      MACM_ST_* bits
  unsigned long long* env_counters;  // [E, 4] per-env accumulators (see macm_world_counters)
  double* env_rsum;              // [E]      per-env reward sum, float64 (macm_world_reward_sums)
  unsigned long long* stamps;    // [E, 16] diagnostic build only (MACM_STAMPS), else NULL
  float2* scratch;               // [E, tcap] list-order impulses (workgroup kernel only)
  // Workgroup path, split step (flock_step_wg_a -> flock_solve_wg -> flock_step_wg_c), per env:
  float4* x_cst;                 // [E, tcap] touching contacts in level order (ab bits, nx, ny, level << 16 | island)
  float2* x_cimp;                // [E, tcap] their impulses (normal, tangent), level order
  uint16_t* x_ord;               // [E, tcap] level order -> touching (list) rank
  uint16_t* x_ic;                // [E, IS]   island contact ranges (IS = N/2 + 2)
  int32_t* x_nlvl;               // [E]       number of Gauss-Seidel levels (diagnostics)
  uint16_t* x_ib;                // [E, IS]   island body ranges
  uint16_t* x_ibod;              // [E, N]    island bodies
  int32_t* x_nisl;               // [E]
  float2* x_vmid;                // [E, N]    velocities after integration (solver input)
  float2* x_cout;                // [E, N]    positions after the position solve
  float2* x_vout;                // [E, N]    velocities after the solve (max-translation clamped)
  uint8_t* x_deg;                // [E, N]    body has touching edges
  uint8_t* x_isolv;              // [E, IS]   island position-solved
  // Dense envs' island DFS in its own kernel (flock_dfs_wg): kernel A hands over
  uint32_t* x_tab;               // [E, tcap] touching contacts in list order (a | b << 16)
  uint32_t* x_adj;               // [E, 2 tcap] CSR edges: touching index | other body << 16
  uint16_t* x_off;               // [E, N + 1] CSR offsets ([N] = 2 T)
  uint32_t* x_dfs;               // [E, tcap] island order: CSR edge slot (x_adj) | level << 16
  // Spill step (flock_spill.hpp): HBM working set for envs whose touching contacts exceed the fast
  // kernels' LDS capacities, capacity C = max_contacts per slot (touching contacts are in the list).
  // S slots: S = E (slot = env) when the memory budget allows, else a pool that a spilling env
  // takes a slot of for the duration of its spill step (sp_lock, see spill::acquire_slot).
  uint32_t* sp_tab;              // [S, C]    touching contacts in list order (bit 31: DFS visited)
  uint32_t* sp_adj;              // [S, 2C]   CSR edges (touching-contact indices)
  uint32_t* sp_ord;              // [S, C]    island order -> touching index
  float4* sp_cst;                // [S, C]    island-ordered records (ab bits, nx, ny, 0)
  float2* sp_cim;                // [S, C]    their impulses
  float2* sp_lam;                // [S, C]    list-order impulses of the touching contacts
  void* sp_rec;                  // [S, N]    pair-sweep records (48 B) when not in LDS (N > 64)
  uint32_t* sp_lock;             // [S]       pool: 0 free, 1 taken; NULL: one slot per env
  int32_t sp_pool;               // pool size S (0: one slot per env, slot = env)
  uint32_t* spill_count;         // [E]       steps taken by the spill step (macm_world_spilled)
  uint32_t* host_status;         // mapped pinned host word: nonzero once any env set a status bit
  // [E] the env order of a launch, heaviest first (flock_step_w64.hip, rollout_sched): wave-kernel
  // rollouts, and the workgroup step's kernels (flock_step_wg.hip, wg_env)
  uint32_t* sched;
};

// The B -> C handoff of the workgroup step (flock_step_wg.hip, round 5). Kernel C of a step used to
// start when kernel B's deepest env had finished, while most CUs idled through B's tail. With a
// handoff, kernel C runs on a second stream, launched once every wave of B has started (behind a
// watcher kernel that waits for b_started to reach the step's count, so B is wholly resident first
// and no C block can take the resources a B wave still needs): each B wave publishes its env when it has finished
// (its outputs for C stored write-through, st_wt, and drained first), and C's blocks take the envs
// in that order. q == NULL: no handoff (C's block b steps env order[b]).
struct Handoff {
  unsigned long long* b_started;  // +1 per B wave at its start (monotonic; flock_step_wg.hip wait_count)
  unsigned int* ctr;              // [2] envs B published, envs C took (zeroed by the step's order kernel)
  unsigned long long* q;          // [E] B's finish order: tag << 32 | env
  unsigned int tag;               // this step's tag (entries of earlier steps carry earlier tags)
};

// Write-through (sc1) stores and loads of the bytes kernel B hands to kernel C (the Handoff): agent-scope
// relaxed atomics, which gfx950 issues as global_store / global_load ... sc1. Stored sc1 by every lane,
// drained (vmcnt 0) before the flag, and loaded sc1 after the flag, they need no agent-scope
// release / acquire (MI355X guide, inter-workgroup visibility: a release fence writes back the
// XCD's whole L2, ~2-6 us, and one per B wave serialised in each XCD).
__device__ __forceinline__ void st_wt(float2* p, float2 v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_wt(const float2* p) {
  const unsigned long long w =
      __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((unsigned int)w), __uint_as_float((unsigned int)(w >> 32)));
}
// The tail observation's control words (flock_step_w64.hip TailObs): per launch-tag parity kTailQ row
// counters, each in a 128-B line of its own, then one ready word per env
constexpr int kTailQ = 64, kTailLine = 16;
__host__ __device__ constexpr size_t tail_ctl_words(int n_envs) { return 2 * kTailQ * kTailLine + (size_t)n_envs; }

__device__ __forceinline__ void st_wt4(float4* p, float4 v) {
  st_wt(reinterpret_cast<float2*>(p), make_float2(v.x, v.y));
  st_wt(reinterpret_cast<float2*>(p) + 1, make_float2(v.z, v.w));
}
__device__ __forceinline__ float4 ld_wt4(const float4* p) {
  const float2 a = ld_wt(reinterpret_cast<const float2*>(p)), b = ld_wt(reinterpret_cast<const float2*>(p) + 1);
  return make_float4(a.x, a.y, b.x, b.y);
}
__device__ __forceinline__ void st_wt(uint8_t* p, uint8_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint8_t ld_wt(const uint8_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(uint16_t* p, uint16_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint16_t ld_wt(const uint16_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_wt(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Host side of a world's handoff (macm_capi.hip): kernel C's stream, the join event, the device
// words of Handoff, the last step's tag and the b_started count the next step waits for.
struct HandoffStream {
  hipStream_t stream;
  hipEvent_t done;
  hipEvent_t pre_b;  // recorded on the caller's stream just before kernel B: the watcher's stream waits on it
  unsigned long long* b_started;
  unsigned int* ctr;
  unsigned long long* q;
  unsigned int tag;
  unsigned long long expected;
};

// A status bit was set in some env: tell the host without a synchronisation (macm_world_step
// reads the word before each launch). Rare path; a plain store, so bits of different envs may
// overwrite each other (the per-env B.status keeps the exact OR for macm_world_status).
__device__ __forceinline__ void report_status(const WorldBuffers& B, int st) {
  if (B.host_status) __hip_atomic_store(B.host_status, (uint32_t)st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Env modes of the wave-per-env kernel: same physics, different env layer.
enum EnvMode : int { kFlock = 0, kTdm = 1 };

// TDM env constants (gym_macm/envs/combat.py:13-49, combatSettings settings.py:149-177).
struct TdmParams {
  int32_t n_teams;
  int32_t team_end[4];          // agent i is in team t iff team_end[t-1] <= i < team_end[t]
  int32_t fresh_raycast;        // 0: the reference's shared, never-reset listener (literal)
  int32_t decay_mov_penalty;    // 0: cooldown_mov_penalty never decrements (literal)
  int32_t _pad;
  double melee_range;           // 2
  double melee_dmg;             // 0.25
  double cooldown_atk;          // 1
  double cooldown_mov_penalty;  // 0.5
  double percent_mov_penalty;   // 0.2
  double init_health;           // 1
};

struct TdmBuffers {
  double* health;        // [E, N]
  double* cd_atk;        // [E, N]
  double* cd_mov;        // [E, N]
  uint8_t* alive;        // [E, N]
  int2* listener;        // [E]  (RayCastClosestCallback.hit, body of .fixture or -1)
  int32_t* winner;       // [E]  -1 = none
  // optional per-step outputs (NULL = not wanted)
  uint8_t* mask_out;     // [E, N, N-1]
  double* health_out;    // [E, N]
  uint8_t* alive_out;    // [E, N]
  int32_t* winner_out;   // [E]
  // the split observation (round 6, tdm_obs_snap.hip): non-NULL, the step writes each agent's pose
  // after the step here, (x, y, angle, alive ? 1 : 0), instead of the observation, and
  // tdm_observe_snap writes the observation and mask from it in a launch of its own
  float4* snap_out;      // [E, N]
};

__host__ __device__ inline int tdm_team_of(const TdmParams& T, int i) {
  int t = 0;
  while (t < T.n_teams - 1 && i >= T.team_end[t]) ++t;
  return t;
}

// sin/cos of the action angle and of angle + pi/2 (mvmnt.py:113-116, combat.py:147):
// macm_action_trig (macm_math.h; its derived float32 forces and ray offsets equal glibc's
// for every float32 angle |a| < 2^19, tools/trig_check.c) in that range, the device libm
// beyond it (|angle| >= 2^19 only arises from injected state: the step wraps into [-pi, pi]).
__device__ __forceinline__ void act_trig(float a, double* s0, double* c0, double* s1, double* c1) {
  if (fabsf(a) < 524288.0f) {
    macm_action_trig(a, s0, c0, s1, c1);
  } else {
    sincos((double)a, s0, c0);
    sincos((double)a + M_PI / 2, s1, c1);
  }
}

// sqrt((double)x) of a float32 x (b2DistanceSquared), as stored into an OT observation.
// For float32 outputs the correctly rounded sqrtf (HIP's default lowering) equals
// (float)sqrt((double)x): double rounding is innocuous for sqrt since 53 >= 2 * 24 + 2
// (device check over every float32: tools/sqrt_gpu_check.hip). Much cheaper than the f64
// sequence.
template <typename OT>
__device__ __forceinline__ double obs_sqrt(float x) {
  if constexpr (sizeof(OT) == 4) return (double)sqrtf(x);
  else return sqrt((double)x);
}

// Correctly rounded 1.0f / x and sqrtf(x) in fewer instructions than HIP's default lowering,
// for the contact normal (b2Vec2::Normalize), which sits on the serial position-solve chain.
// rcp_rn: v_rcp_f32 plus one fma Newton step; equals 1.0f / x for every float32 x in
// [2^-23, 2^64] (Normalize only divides by len >= FLT_EPSILON; len <= sqrt(FLT_MAX) < 2^64).
// sqrt_rn: v_sqrt_f32 with the +-1 ulp residual correction of the default lowering but
// without its denormal scaling; equals sqrtf(x) for every float32 x >= 2^-48, and below
// that both results are < FLT_EPSILON, so Normalize takes the same branch.
// Both checked on the device over every float32 input (tools/rcp_sqrt_gpu_check.hip).
__device__ __forceinline__ float rcp_rn(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, y, 1.0f);
  return __builtin_fmaf(e, y, y);
}

__device__ __forceinline__ float sqrt_rn(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __uint_as_float(__float_as_uint(s) - 1u);
  const float su = __uint_as_float(__float_as_uint(s) + 1u);
  float r = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
  r = __builtin_fmaf(-su, s, x) > 0.0f ? su : r;
  return r;
}

// RN(n / K) for a loop-invariant K > 0 (the position solve's -C / (mA + mB)) from rK = RN(1 / K),
// hoisted out of the loop: q0 = n * rK is within a few ulps, one fma correction makes it
// faithful and a second is Markstein's correction step, which returns the correctly rounded
// quotient for a faithful one and rK = RN(1 / K), away from underflow. Here n = -b2Clamp(0.2f *
// fl(sep + 0.005f), -0.2f, 0) is 0 or >= 2^-35: a nonzero fl(sep + 0.005f) is >= 0.0025 in
// magnitude unless sep is in (-0.01, -0.0025), where the sum is exact (Sterbenz) and a multiple
// of ulp(0.0025) = 2^-32. Checked on the device for every float32 n in {0} u [2^-40, 0.2] and K of
// the default and 255 random configs: 0 mismatches (tools/rcp_sqrt_gpu_check.hip; below 2^-40
// the sequence can differ, and is never given such n).
__device__ __forceinline__ float div_by_invariant(float n, float K) {
  const float rK = 1.0f / K;
  const float q0 = n * rK;
  const float q1 = __builtin_fmaf(__builtin_fmaf(-K, q0, n), rK, q0);
  // the sign of the quotient is the sign of n (K > 0); copysign keeps it for n = -0, where the
  // fma corrections would return +0 and n / K gives -0 (the sign can reach a zero position)
  return __builtin_copysignf(__builtin_fmaf(__builtin_fmaf(-K, q1, n), rK, q1), n);
}

// Between the level steps of a one-wave Gauss-Seidel solve: the next step's lanes read the body
// updates this step's lanes wrote to LDS. A wave's LDS accesses are performed in issue order, so
// wavefront-scope release/acquire fences (no wait) are enough: the reads are issued after the
// writes and cannot pass them. Waiting for the writes to complete (lgkmcnt(0), the round-2
// first version) added an LDS round trip to every level step.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive prefix maximum over the 64 lanes of a wave in lane order, by DPP row shifts and row
// broadcasts (no LDS crossbar round trips). Values must be > -2^30 (the identity used).
// The whole wave must be active. Each step is one v_max_i32 with a DPP source: a lane whose source
// is out of its row (no bound_ctrl) or outside the row mask is not written and keeps its own value,
// which is the maximum's identity there. The compiler does not fold update_dpp into the max (it
// emits a mov_dpp, an identity mov and the max per step: 24 instructions against 12).
__device__ __forceinline__ int wave_prefix_max(int v) {
  asm volatile(
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(v));
  return v;
}

// Inclusive prefix sum over the 64 lanes of a wave in lane order (integers), the DPP form of
// wave_prefix_max: a lane whose DPP source is outside its row or the row mask is not written and
// keeps its own partial sum. The whole wave must be active (__shfl_up steps: six LDS-crossbar
// round trips).
__device__ __forceinline__ int wave_prefix_sum(int v) {
  asm volatile(
      "s_nop 1\n\t"
      "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(v));
  return v;
}

// Stores of the Flock step's per-agent outputs (obs, reward, neighbour id, collided): nontemporal
// (the policy reads them, the step does not): driver window 34.0 -> 33.5 us, steady 21.6 -> 21.4 us
// (profiles/r02/nt_stores). Not for TDM's [E, N, N-1, 4] obs: its 16-byte pair-tile stores then
// stop combining in L2 (C4 32.3 -> 62.5 us). Nor for the state and contact list the next step
// reads (no gain).
template <int KIND, typename T>
__device__ __forceinline__ void st_g(T* p, const T& v) {
  constexpr bool nt = KIND == 0;
  if constexpr (nt) {
    if constexpr (sizeof(T) == 16) {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      v4u x;
      __builtin_memcpy(&x, &v, 16);
      __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
    } else if constexpr (sizeof(T) == 8) {
      unsigned long long x;
      __builtin_memcpy(&x, &v, 8);
      __builtin_nontemporal_store(x, reinterpret_cast<unsigned long long*>(p));
    } else if constexpr (sizeof(T) == 4) {
      unsigned int x;
      __builtin_memcpy(&x, &v, 4);
      __builtin_nontemporal_store(x, reinterpret_cast<unsigned int*>(p));
    } else {
      __builtin_nontemporal_store(v, p);
    }
    return;
  }
  *p = v;
}
constexpr int kOut = 0, kState = 1;

__device__ __forceinline__ int wave_max(int v) {  // over all 64 lanes, wave-uniform
  return __builtin_amdgcn_readlane(wave_prefix_max(v), 63);
}

// ---- the reward sum (macm_world_reward_sums) -----------------------------------
// One env-step's rewards are summed as float64 values of the float32 rewards the step writes, in a
// fixed order, so the per-env total is bit-stable and the host restates it exactly
// (gym_macm.dist.pairwise_reward_sum): pairwise over the agent slots 0 .. P - 1 with +0.0 in the
// slots of lanes >= N, P = 64 * 2^ceil(log2(waves of the block)). That is an xor butterfly within a
// wave — lane 0 holds ((r0 + r1) + (r2 + r3)) + ... — and the waves' sums pairwise in the same way.
// Each level here pairs partial sums whose pairing equals the xor butterfly's (every lane of a group
// holds its group's sum once the level before has run; IEEE addition is commutative), by DPP
// within rows and lane reads across them, with no LDS round trip.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Pairwise sum of the wave's 64 values (the whole wave active); wave-uniform result.
__device__ __forceinline__ double wave_pairwise_sum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1, 0, 3, 2]: r0 + r1
  v += dpp_f64<0x4E>(v);   // quad_perm [2, 3, 0, 1]: (r0 + r1) + (r2 + r3)
  v += dpp_f64<0x141>(v);  // row_half_mirror: lane i <- 7 - i, the other quad's sum
  v += dpp_f64<0x140>(v);  // row_mirror: lane i <- 15 - i, the other half-row's sum
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}
// The same over a block of blockDim.x / 64 <= 16 waves (every thread calls it; s_tmp: 16 doubles of
// LDS, free on entry and on return); the result is valid in thread 0.
__device__ __forceinline__ double block_pairwise_sum(double v, double* s_tmp) {
  v = wave_pairwise_sum(v);
  const int nw = blockDim.x >> 6, wid = threadIdx.x >> 6;
  if (nw == 1) return v;
  if ((threadIdx.x & 63) == 0) s_tmp[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int n2 = 1;
    while (n2 < nw) n2 <<= 1;
    for (int q = nw; q < n2; ++q) s_tmp[q] = 0.0;
    for (int h = 1; h < n2; h <<= 1)
      for (int q = 0; q + h < n2; q += 2 * h) s_tmp[q] = s_tmp[q] + s_tmp[q + h];
    v = s_tmp[0];
  }
  __syncthreads();
  return v;
}

// env e's total += one step's sum, as a float64 atomic add without return: the wave does not wait
// for it (a load-add-store held 2 VGPRs across the step's observation and spilled in the rollout
// kernel) and the adds of one wave to one address take effect in program order (per-location
// coherence), so the total is the steps' sums added in step order. No denormal arises (the sums are
// of float32 rewards in [-1, 1]). Every writer of env_rsum uses it.
__device__ __forceinline__ void add_reward_sum(const WorldBuffers& B, int e, double v) {
  unsafeAtomicAdd(B.env_rsum + e, v);
}

// Per-env CPython MT19937 streams in HBM for device-side resets (csrc/env_reset.hip).
constexpr int kMtStride = 640;  // words per env: 624 state words, [624] = position

struct PoseDraw {
  int mode;  // kFlock / kTdm
  int n_agents;
  double spread, start_x, start_y;  // Flock (flockSettings start_spread / start_point)
  double half_width, height;        // TDM (world_width / 2, world_height)
  TdmParams TP;                     // TDM team boundaries
};

}  // namespace macm
