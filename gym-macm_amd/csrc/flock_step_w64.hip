// flock_step_w64.hip — batched Flock / TDM env.step for N <= 64 agents per env on gfx950.
//
// One 64-lane wavefront advances one env; lane i owns agent i. Per-env state is
// staged in registers + LDS (< 10 KB, so 16 envs fit a CU and a 4096-env step is
// one dispatch round) and written back once. The step restates, in one launch:
//   action -> angle/force                gym_macm/envs/mvmnt.py:97-129
//   b2World::Step(1/hz, 8, 3)            gym_macm/cm_framework.py:222-223 [EXT-B2D]
//     Collide (contact persistence, circle manifolds, warm-start carry)
//     island DFS in Box2D order, integrate velocities + damping,
//     sequential-impulse velocity solve (warm start + 8 iterations),
//     integrate positions, position solve (<= 3 iterations, early exit),
//     sleep, SynchronizeFixtures (fat-AABB hysteresis), FindNewContacts
//   ClearForces                           cm_framework.py:224
//   get_rewards                           mvmnt.py:160-179
//   time / done                           mvmnt.py:134-136
//   get_obs                               mvmnt.py:181-222
//
// Box2D-order representation. Box2D keeps contacts in a world list and per-body
// edge lists, both prepend-on-create; its island DFS walks bodies in reverse
// creation order and each body's edges most-recent-first, and the Gauss-Seidel
// sweep follows that order. Here each env carries ONE ordered array of the
// contacts that survive the next Collide (the pairs whose current fat AABBs
// overlap): each step prepends the newly created pairs in descending (a, b)
// order (FindNewContacts sorts pairs ascending and prepends each) and keeps the
// surviving old pairs in their order. A body's edge list is then this array
// restricted to the body's contacts, so the DFS below visits contacts in exactly
// Box2D's order and the solver reproduces Box2D's rounding sequence.
//
// Where the time goes (tools/phase_profile.py, tools/timeline.py, profiles/r01/): the
// step is latency-bound, not bandwidth-bound, and its duration is that of the envs with
// the most touching contacts, whose serial Box2D chain (island DFS, Gauss-Seidel, position
// passes) outlasts the other waves. Hence: every global load the step needs is issued up
// front; list entries and their impulses arrive in one round trip and stay in registers;
// the chain runs at raised issue priority (s_setprio), the DFS walks scalar bit masks
// through v_readlane / v_writelane, small islands keep their records in registers, and
// bodies sit in LDS as float2; the all-pairs sweep reads records by LDS broadcast in two
// interleaved chains; per-env counters instead of global atomics.
//
// Exactness notes (checked by tests/test_gpu_parity.py against the oracle):
//   * fixedRotation bodies have invI = 0 and w = 0, so every angular term in the
//     solver is a signed zero; dropping them can change only the sign of a zero
//     velocity/impulse component, never a nonzero value or any position.
//   * circles sit at the body origin, so b2Mul(xf, m_p) == position exactly.
#include "bots.hpp"
#include "flock_common.hpp"
#include "flock_spill.hpp"
#include "tdm_obs.hpp"

namespace macm {

constexpr int W = 64;       // wavefront = one env's agent lanes
// touching contacts per env held in LDS (indices fit uint8); more take the spill step. With s_adj
// aliased onto s_tm and the sweep records over s_tn + s_tab the Flock kernel needs 8.3 KB of LDS:
// 19 waves per CU, so a 4096-env launch (16 per CU) has slack (at 16 per CU, -4% per step at M
// and -7% in the bots closed loop; TCAP 224 fits 20 per CU but sends dense bots envs to the
// spill step: profiles/r02/wave_levels)
constexpr int TCAP = 256;
constexpr int DEG = 16;     // touching contacts per body
constexpr int ICAP = W / 2; // islands with >= 1 contact (>= 2 bodies each)
constexpr int RCH = 2;      // list chunks (of 64 entries) cached in registers
// Islands of 2..KREC contacts keep their contact records (pair, normal) and impulses in
// registers for the whole velocity / position solve; only the bodies' velocities and
// positions go through LDS, so a contact update waits on one LDS round trip instead of
// three (order -> record -> bodies). Measured -3.3% per step at the metric config
// (profiles/r01/ab2). Keeping the bodies in registers too (per-contact copies, forwarded
// after every update) was slower: +6% at 2..3 contacts.
constexpr int KREC = 4;
constexpr int KRECA = KREC;
// In a wave that has 2..KREC-contact islands, its single-contact islands join the same
// register-record solve (as islands of one contact) instead of running their own register
// loop before it: the wave then walks max-island-size x 9 updates instead of 9 more on top
// (single-contact lanes pay the LDS round trip that the multi-contact lanes wait on anyway).
// Gauss-Seidel levels (T <= 64 touching contacts): the scalar DFS also gives each contact its
// level, 1 + the level of the last earlier contact (island order) sharing a body with it; lane k
// holds the k-th contact's record and the wave solves a level's contacts together (they share no
// body, so every body keeps Box2D's sequence of updates). The level path runs when an island has
// more than kLevelsMinIsland contacts (the register-record islands take the rest).
constexpr int kLevelsMinIsland = 4;
constexpr int kPrio2T = 3;  // touching contacts from which a wave keeps priority 2 after the chain
// TDM obs in row-block order with the transposed half staged (tdm_obs.hpp tdm_obs_rowblocks, round 4;
// float32 obs, N <= 32: the 6 KB stage), else the pair tiles (tdm_obs_pairs). Measured and dropped
// (round 6 removed their code; evidence kept): the staged memory-order writer, 709 B per agent-step
// of HBM traffic instead of 864 but C4 34.1 us per step instead of 28.2 (profiles/r03/abtests/tdm_obs/);
// the mask staged in LDS, time unchanged with more scratch (profiles/r04/tdm_mask/).

// Diagnostic build only (-DMACM_STAMPS, build/libmacm_hip_stamps.so via `make stamps`):
// lane 0 records s_memtime at phase boundaries into B.stamps[e][0..13] and per-env
// sizes into [14..15]. The product library compiles these to nothing.
// -DMACM_TIMELINE (with MACM_STAMPS for the buffer): instead of phase stamps, lane 0
// records only [0] s_memrealtime and [1] s_memtime at entry, [2] HW_ID | XCC_ID << 32,
// [3] / [4] the same clocks after the last store is issued (tools/timeline.py).
#if defined(MACM_STAMPS) && !defined(MACM_TIMELINE)
#define STAMP(k)                                                                    \
  do {                                                                              \
    __builtin_amdgcn_s_waitcnt(0);                                                  \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                     \
    if (lane == 0) B.stamps[(size_t)e * 16 + (k)] = _t;                             \
  } while (0)
#define STAMP_STAT(k, v)                                                            \
  do {                                                                              \
    if (lane == 0) B.stamps[(size_t)e * 16 + (k)] = (unsigned long long)(v);        \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#define STAMP_STAT(k, v) \
  do {                   \
  } while (0)
#endif

__device__ __forceinline__ float bmin(float a, float b) { return a < b ? a : b; }  // b2Min
__device__ __forceinline__ float bmax(float a, float b) { return a > b ? a : b; }  // b2Max
// The contact solvers' clamps as single v_min_f32 / v_max_f32 instead of compare + select
// (b2Min / b2Max): they sit on the serial Gauss-Seidel chain. For non-NaN operands the two
// forms differ only in the sign of a zero result (b2Max(-0, +0) is +0, v_max may give -0);
// a zero impulse or velocity of either sign leaves every later value the same, so only
// zero signs can differ (as they already do through the angular terms).
// sclamp as one v_med3_f32: the median of (a, lo, hi) is the clamp for lo <= hi and non-NaN a.
__device__ __forceinline__ float smax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ float sclamp(float a, float lo, float hi) { return __builtin_amdgcn_fmed3f(a, lo, hi); }

// b2TestOverlap
__device__ __forceinline__ bool overlap(float4 a, float4 b) {
  const float d1x = b.x - a.z, d1y = b.y - a.w;
  const float d2x = a.x - b.z, d2y = a.y - b.w;
  if (d1x > 0.0f || d1y > 0.0f) return false;
  if (d2x > 0.0f || d2y > 0.0f) return false;
  return true;
}

// b2Vec2::Normalize (sqrt_rn / rcp_rn: the correctly rounded sqrtf and 1.0f / len, flock_common.hpp)
__device__ __forceinline__ void normalize(float& x, float& y) {
  const float len = sqrt_rn(x * x + y * y);
  if (len < kEps) return;
  const float inv = rcp_rn(len);
  x *= inv;
  y *= inv;
}

// v_writelane_b32 with a wave-uniform lane index (in M0: on gfx9 the lane select and the
// data cannot both be SGPRs): lane `l` of v receives the uniform value x. The s_nop covers
// the SALU write of M0 just before.
__device__ __forceinline__ uint32_t writelane_m0(int x, int l, uint32_t v) {
  // x and l are wave-uniform; readfirstlane makes that visible where the compiler cannot
  // prove it (an SGPR operand)
  asm volatile("s_nop 1\n\tv_writelane_b32 %0, %1, m0"
               : "+v"(v)
               : "s"(__builtin_amdgcn_readfirstlane(x)), "{m0}"(__builtin_amdgcn_readfirstlane(l)));
  return v;
}

// the number of set bits of m below this lane (v_mbcnt)
__device__ __forceinline__ int mbcnt64(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) {
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

typedef float fvec2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fvec2 mk2(float a, float b) {
  fvec2 v;
  v.x = a;
  v.y = b;
  return v;
}

// One agent's record for the all-pairs sweep: read by LDS broadcast (2 x ds_read_b128).
struct __align__(32) PairRec {
  float4 fn;  // fat AABB after SynchronizeFixtures
  float2 c;   // final position
  float2 pad;
};

// v_readlane with a wave-uniform lane index: broadcast without an LDS round trip.
__device__ __forceinline__ float bcast(float v, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

template <typename OT>
__device__ __forceinline__ void write_obs_row(OT* o, int coord, double r0, double t0, double r1, double t1) {
  if (coord == MACM_COORD_CARTESIAN) {
    o[0] = (OT)r0;
    o[1] = (OT)cos(t0);
    o[2] = (OT)sin(t0);
    o[3] = (OT)r1;
    o[4] = (OT)cos(t1);
    o[5] = (OT)sin(t1);
  } else if constexpr (sizeof(OT) == 4) {
    st_g<kOut>(reinterpret_cast<float4*>(o), make_float4((float)r0, (float)t0, (float)r1, (float)t1));
  } else {
    st_g<kOut>(reinterpret_cast<double2*>(o), make_double2(r0, t0));
    st_g<kOut>(reinterpret_cast<double2*>(o) + 1, make_double2(r1, t1));
  }
}

// Flock.get_obs for one agent (mvmnt.py:181-222): node 0 = closest other agent
// (squared distance `best`, relative position (rx, ry) = other - self, float32),
// node 1 = the agent's target (relative position target - self, float32).
template <typename OT>
__device__ __forceinline__ void write_obs(OT* o, int coord, float ang, float best, float rx, float ry, float tdx,
                                          float tdy, float td2) {
  // obs_atan2 (macm_math.h): <= 1 ulp from glibc atan2 in f64, identical after "- angle"
  // and the float32 rounding (tools/atan2_check.c), about half the device libm's work
  const double t0 = wrap_pi(obs_atan2((double)ry, (double)rx) - (double)ang);
  const double t1 = wrap_pi(obs_atan2((double)tdy, (double)tdx) - (double)ang);
  write_obs_row(o, coord, obs_sqrt<OT>(best), t0, obs_sqrt<OT>(td2), t1);
}

// The same two functions on (x, y) pairs: v_pk_mul_f32 / v_pk_add_f32 are, lane by lane, the
// scalar form's IEEE operations (no contraction: -ffp-contract=off), so results are bit-identical;
// the dependent chain is ~1/3 shorter (tools/ubench_level.hip V6 vs V1: 287 vs 307 cycles per level
// step for a wave alone on its SIMD, 293 vs 311 at two waves per SIMD, 389 vs 381 at four).
typedef float pf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void warm_start_contact_pk(pf2& vA, pf2& vB, float nx, float ny, float ln, float ltg,
                                                      float mA, float mB) {
  const pf2 n = {nx, ny}, t = {ny, -nx};
  const pf2 P = ln * n + ltg * t;
  vA = vA - mA * P;
  vB = vB + mB * P;
}

__device__ __forceinline__ void solve_velocity_contact_pk(pf2& vA, pf2& vB, float nx, float ny, float& ln,
                                                          float& ltg, float mA, float mB, float kmass,
                                                          float friction) {
  const pf2 n = {nx, ny}, t = {ny, -nx};
  {  // tangent first
    const pf2 pr = (vB - vA) * t;
    const float vt = pr.x + pr.y;
    float lambda = kmass * (-vt);
    const float maxf = friction * ln;
    const float ni = sclamp(ltg + lambda, -maxf, maxf);
    lambda = ni - ltg;
    ltg = ni;
    const pf2 P = lambda * t;
    vA = vA - mA * P;
    vB = vB + mB * P;
  }
  {  // normal
    const pf2 pr = (vB - vA) * n;
    const float vn = pr.x + pr.y;
    float lambda = -kmass * (vn - 0.0f);
    const float ni = smax(ln + lambda, 0.0f);
    lambda = ni - ln;
    ln = ni;
    const pf2 P = lambda * n;
    vA = vA - mA * P;
    vB = vB + mB * P;
  }
}

// The chains outside the wide levels (one-slot levels, per-island lanes, single contacts) stay on
// scalar components: on packed pairs they measured slower (round 5, profiles/r05/abtests/).

// b2ContactSolver, one circle contact (fixedRotation: no angular terms). Shared by
// the LDS path and the single-contact register path, so both round identically.
__device__ __forceinline__ void warm_start_contact(float& vAx, float& vAy, float& vBx, float& vBy, float nx,
                                                   float ny, float ln, float ltg, float mA, float mB) {
  const float tx = ny, ty = -nx;  // b2Cross(normal, 1.0f)
  const float Px = ln * nx + ltg * tx, Py = ln * ny + ltg * ty;
  vAx = vAx - mA * Px;
  vAy = vAy - mA * Py;
  vBx = vBx + mB * Px;
  vBy = vBy + mB * Py;
}

__device__ __forceinline__ void solve_velocity_contact(float& vAx, float& vAy, float& vBx, float& vBy, float nx,
                                                       float ny, float& ln, float& ltg, float mA, float mB,
                                                       float kmass, float friction) {
  const float tx = ny, ty = -nx;
  {  // tangent first
    const float dvx = vBx - vAx, dvy = vBy - vAy;
    const float vt = dvx * tx + dvy * ty;
    float lambda = kmass * (-vt);
    const float maxf = friction * ln;
    const float ni = sclamp(ltg + lambda, -maxf, maxf);
    lambda = ni - ltg;
    ltg = ni;
    const float Px = lambda * tx, Py = lambda * ty;
    vAx = vAx - mA * Px;
    vAy = vAy - mA * Py;
    vBx = vBx + mB * Px;
    vBy = vBy + mB * Py;
  }
  {  // normal
    const float dvx = vBx - vAx, dvy = vBy - vAy;
    const float vn = dvx * nx + dvy * ny;
    float lambda = -kmass * (vn - 0.0f);  // velocityBias == 0 (restitution 0)
    const float ni = smax(ln + lambda, 0.0f);
    lambda = ni - ln;
    ln = ni;
    const float Px = lambda * nx, Py = lambda * ny;
    vAx = vAx - mA * Px;
    vAy = vAy - mA * Py;
    vBx = vBx + mB * Px;
    vBy = vBy + mB * Py;
  }
}

__device__ __forceinline__ float solve_position_contact_pk(pf2& cA, pf2& cB, float radius, float mA, float mB) {
  const pf2 d = cB - cA;
  const pf2 d2 = d * d;
  const float len = sqrt_rn(d2.x + d2.y);
  const pf2 n = len < kEps ? d : d * rcp_rn(len);  // b2Vec2::Normalize
  const pf2 pr = d * n;
  const float sep = (pr.x + pr.y) - radius - radius;
  const float Cc = sclamp(kBaumgarte * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
  const float K = mA + mB;
  const float imp = K > 0.0f ? div_by_invariant(-Cc, K) : 0.0f;
  const pf2 P = imp * n;
  cA = cA - mA * P;
  cB = cB + mB * P;
  return sep;
}

// b2PositionSolverManifold + one SolvePositionConstraints contact; returns sep.
__device__ __forceinline__ float solve_position_contact(float& cAx, float& cAy, float& cBx, float& cBy,
                                                        float radius, float mA, float mB) {
  float nx = cBx - cAx, ny = cBy - cAy;
  normalize(nx, ny);
  const float sep = ((cBx - cAx) * nx + (cBy - cAy) * ny) - radius - radius;
  const float Cc = sclamp(kBaumgarte * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
  const float K = mA + mB;
  const float imp = K > 0.0f ? div_by_invariant(-Cc, K) : 0.0f;
  const float Px = imp * nx, Py = imp * ny;
  cAx = cAx - mA * Px;
  cAy = cAy - mA * Py;
  cBx = cBx + mB * Px;
  cBy = cBy + mB * Py;
  return sep;
}

template <bool B>
struct BoolC {
  static constexpr bool value = B;
};
template <int I>
struct IntC {
  static constexpr int value = I;
};

// Gauss-Seidel levels for 64 < T <= TCAP touching contacts (round 3): contact k of the island
// order sits in slot k / 64 of lane k % 64 (S = 2 slots up to 128 contacts, 4 up to 256). Levels as
// in the one-slot path: level(k) = 1 + the level of the last earlier contact sharing a body with k,
// from one scalar walk in island order, so the contacts of a level share no body and every body
// takes Box2D's sequence of updates. A level step is branch-free until its stores: every slot
// reads its two bodies and solves (the S chains interleave), and only the slots of the current
// level store bodies (exec-masked) and keep their impulses.
constexpr int kNoLevel = 0xffff;  // a slot without a contact (or whose island has left the passes)
// One-slot level steps: the lanes outside the level on a dummy slot each (round 3; one shared slot
// measured M bots +2%, profiles/r04/abtests/shared_dummy/). The wide levels' updates run on packed
// pairs (round 5: M closed loop -2.6%, metric window -0.5%, profiles/r05/abtests/wide_packed/).
// Measured slower and removed in round 6 (evidence kept): skipping a wide slot by its level range
// (M bots 161 -> 197 us, profiles/r04/abtests/serial_prefetch/), slots in island order, the island
// walk a popped body at a time (par_dfs), the wide position minima in registers, priority 3 for the
// wide-level waves only.

// S slots per lane; REG: each slot's normal and impulses in registers (S = 2, T <= 128), else read
// from / written to the touching-contact arrays in LDS at every level step (S = 4: registers for
// four slots would push the kernel past 96 VGPRs, i.e. below 5 waves per SIMD, for every env)
struct WideLevels {
  uint32_t pw[4];      // a | b << 8 | t << 16 (t: touching (list) rank)
  uint32_t lvis[4];    // level (kNoLevel if none) | island << 16
  float nx[4], ny[4];  // REG: normal
  float ln[4], lt[4];  // REG: accumulated normal / tangent impulse
  int dmax;            // number of levels (wave-uniform)

  __device__ __forceinline__ static int ia(uint32_t w) { return w & 0xffu; }
  __device__ __forceinline__ static int ib(uint32_t w) { return (w >> 8) & 0xffu; }
  __device__ __forceinline__ static int it(uint32_t w) { return w >> 16; }
  __device__ __forceinline__ static int lvl(uint32_t x) { return x & 0xffffu; }
  __device__ __forceinline__ static int isl(uint32_t x) { return x >> 16; }

  template <int S, bool REG>
  __device__ __forceinline__ void init(int lane, int Tw, int nisl, uint8_t* s_ord, const uint32_t* s_tab,
                                       const float* s_tnx, const float* s_tny, const float* s_tln,
                                       const float* s_tlt, const uint16_t* s_ic, uint32_t* s_tmp) {
    uint32_t abq[S];
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const int k = 64 * q + lane;
      const int t = k < Tw ? (int)s_ord[k] : 0;
      const uint32_t ab = k < Tw ? s_tab[t] : 0u;
      abq[q] = (ab & 0xffu) | ((ab >> 8) & 0xff00u);
      pw[q] = abq[q] | ((uint32_t)t << 16);
      if constexpr (REG) {
        nx[q] = s_tnx[t];
        ny[q] = s_tny[t];
        ln[q] = s_tln[t];
        lt[q] = s_tlt[t];
      }
    }
    // levels: scalar walk in island order (lane b of lastv: 1 + the level of the last contact on body b)
    uint32_t lastv = 0u;
    int dm = 0;
#pragma unroll
    for (int q = 0; q < S; ++q) {
      uint32_t lvv = (uint32_t)kNoLevel;
      const int n = min(64, Tw - 64 * q);
      for (int kk = 0; kk < n; ++kk) {
        const uint32_t p = (uint32_t)__builtin_amdgcn_readlane(abq[q], kk);
        const int a = p & 0xffu, b = p >> 8;
        const int l = max(__builtin_amdgcn_readlane(lastv, a), __builtin_amdgcn_readlane(lastv, b));
        lastv = writelane_m0(l + 1, a, lastv);
        lastv = writelane_m0(l + 1, b, lastv);
        lvv = writelane_m0(l, kk, lvv);
        dm = max(dm, l + 1);
      }
      lvis[q] = lvv;
    }
    dmax = dm;
    // island of each contact: the islands whose first contact is at or before it
    const int icv = lane <= nisl ? (int)s_ic[lane] : 0x7fffffff;
    int is[S];
#pragma unroll
    for (int q = 0; q < S; ++q) is[q] = 0;
    for (int I = 1; I < nisl; ++I) {
      const int c = __builtin_amdgcn_readlane(icv, I);
#pragma unroll
      for (int q = 0; q < S; ++q) is[q] += 64 * q + lane >= c ? 1 : 0;
    }
#pragma unroll
    for (int q = 0; q < S; ++q) lvis[q] |= (uint32_t)is[q] << 16;
    reorder<S, REG>(lane, Tw, s_ord, s_tab, s_tnx, s_tny, s_tln, s_tlt, s_tmp);
  }

  // Level order (round 4): contact k of the level-sorted order moves to slot k / 64 of lane k % 64,
  // so a level's contacts fill one slot (a level straddles two slots at most once) and a level step
  // runs one slot's update. In island order every island restarts at level 0, so with two or more
  // islands most level steps ran an update per slot. Contacts of one level share no body: their
  // order within the level changes nothing. s_tmp (>= 512 B, the DFS masks, dead here): the level
  // histogram as 16-bit counters, then each contact's level | island << 8 at its new place.
  template <int S, bool REG>
  __device__ __forceinline__ void reorder(int lane, int Tw, uint8_t* s_ord, const uint32_t* s_tab,
                                          const float* s_tnx, const float* s_tny, const float* s_tln,
                                          const float* s_tlt, uint32_t* s_tmp) {
    for (int w = lane; w < 128; w += 64) s_tmp[w] = 0u;  // 256 levels (dmax <= Tw <= 256)
    wave_lds_sync();
    int rk[S], tq[S];
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const int l = lvl(lvis[q]);
      tq[q] = it(pw[q]);
      rk[q] = 0;
      if (l != kNoLevel) {
        const uint32_t sh = 16u * (uint32_t)(l & 1);
        rk[q] = (int)((atomicAdd(&s_tmp[l >> 1], 1u << sh) >> sh) & 0xffffu);
      }
    }
    wave_lds_sync();
    {  // exclusive scan of the counts: lane L owns levels 4L .. 4L + 3 (two words)
      const uint32_t w0 = s_tmp[2 * lane], w1 = s_tmp[2 * lane + 1];
      const int c0 = (int)(w0 & 0xffffu), c1 = (int)(w0 >> 16), c2 = (int)(w1 & 0xffffu), c3 = (int)(w1 >> 16);
      const int sum = c0 + c1 + c2 + c3;
      const int ex = wave_prefix_sum(sum) - sum;
      wave_lds_sync();
      s_tmp[2 * lane] = (uint32_t)ex | ((uint32_t)(ex + c0) << 16);
      s_tmp[2 * lane + 1] = (uint32_t)(ex + c0 + c1) | ((uint32_t)(ex + c0 + c1 + c2) << 16);
    }
    wave_lds_sync();
    int pos[S];
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const int l = lvl(lvis[q]);
      pos[q] = l != kNoLevel ? (int)((s_tmp[l >> 1] >> (16u * (uint32_t)(l & 1))) & 0xffffu) + rk[q] : -1;
    }
    wave_lds_sync();
    uint16_t* const s_lv = reinterpret_cast<uint16_t*>(s_tmp);
#pragma unroll
    for (int q = 0; q < S; ++q)
      if (pos[q] >= 0) {
        s_ord[pos[q]] = (uint8_t)tq[q];
        s_lv[pos[q]] = (uint16_t)(lvl(lvis[q]) | (isl(lvis[q]) << 8));
      }
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const int k = 64 * q + lane;
      const int t = k < Tw ? (int)s_ord[k] : 0;
      const uint32_t ab = k < Tw ? s_tab[t] : 0u;
      const uint32_t lv = k < Tw ? (uint32_t)s_lv[k] : 0u;
      pw[q] = (ab & 0xffu) | ((ab >> 8) & 0xff00u) | ((uint32_t)t << 16);
      lvis[q] = k < Tw ? ((lv & 0xffu) | ((lv >> 8) << 16)) : (uint32_t)kNoLevel;
      if constexpr (REG) {
        nx[q] = s_tnx[t];
        ny[q] = s_tny[t];
        ln[q] = s_tln[t];
        lt[q] = s_tlt[t];
      }
    }
  }

  // warm start (pass -1) + vel_iters velocity passes, level by level; then (REG) the impulses to
  // s_tln / s_tlt
  template <int S, bool REG>
  __device__ __forceinline__ void velocity(const StepParams& P, float2* s_v, const float* s_tnx, const float* s_tny,
                                           float* s_tln, float* s_tlt, float mA, float mB, float kmass,
                                           float friction) {
    // One slot at a time, and only the slots with a contact of the current level: a contact update
    // is ~35 dependent VALU, issued at one per 4 cycles per wave, so a slot's update costs the same
    // whether or not another slot's runs beside it (measured: two slots interleaved were no faster
    // than one after the other), and levels grow along the island order, so in most level steps
    // one slot is busy. The warm-start pass and the velocity passes are separate loops, so that a
    // level step has no branch before its stores.
    // The update stays exec-masked: run branch-free (every lane on the slot, the idle ones on a dummy)
    // it was 14% slower in the M closed loop, where 4-5 waves per SIMD share the CU's LDS.
    auto pass = [&](auto warm) {
      for (int l = 0; l < dmax; ++l) {
#pragma unroll
        for (int q = 0; q < S; ++q) {
          if (lvl(lvis[q]) == l) {  // exec-masked; a slot with no contact of this level is skipped
            if constexpr (S > 2) asm volatile("" : "+v"(pw[q]));  // LDS addresses not hoisted (VGPRs)
            float cx, cy, nl, nt;
            pf2* const pA = reinterpret_cast<pf2*>(s_v + ia(pw[q]));
            pf2* const pB = reinterpret_cast<pf2*>(s_v + ib(pw[q]));
            pf2 vA = *pA, vB = *pB;
            if constexpr (REG) {
              cx = nx[q];
              cy = ny[q];
              nl = ln[q];
              nt = lt[q];
            } else {
              cx = s_tnx[it(pw[q])];
              cy = s_tny[it(pw[q])];
              nl = s_tln[it(pw[q])];
              nt = s_tlt[it(pw[q])];
            }
            if constexpr (decltype(warm)::value) warm_start_contact_pk(vA, vB, cx, cy, nl, nt, mA, mB);
            else solve_velocity_contact_pk(vA, vB, cx, cy, nl, nt, mA, mB, kmass, friction);
            *pA = vA;
            *pB = vB;
            if constexpr (REG) {
              ln[q] = nl;
              lt[q] = nt;
            } else {
              s_tln[it(pw[q])] = nl;
              s_tlt[it(pw[q])] = nt;
            }
          }
        }
        wave_lds_sync();
      }
    };
    if (P.warm_starting) pass(BoolC<true>{});
    for (int itr = 0; itr < P.vel_iters; ++itr) pass(BoolC<false>{});
    if constexpr (REG) {
#pragma unroll
      for (int q = 0; q < S; ++q) {
        if (lvl(lvis[q]) != kNoLevel) {
          s_tln[it(pw[q])] = ln[q];
          s_tlt[it(pw[q])] = lt[q];
        }
      }
    }
  }

  // position passes level by level; an island leaves after the first pass whose minimum separation
  // (from 0) is >= -3 linearSlop (b2Island::Solve), as in the one-slot level path
  template <int S>
  __device__ __forceinline__ void position(const StepParams& P, int lane, int nisl, float2* s_c, int* s_pmin,
                                           uint8_t* s_isolved, float mA, float mB) {
    const unsigned long long islm = nisl >= 64 ? ~0ull : ((1ull << nisl) - 1ull);
    unsigned long long done = 0ull;
    for (int itr = 0; itr < P.pos_iters && done != islm; ++itr) {
      if (lane < nisl) s_pmin[lane] = __float_as_int(0.0f);
      // an island that has left the passes never returns: its contacts lose their level
#pragma unroll
      for (int q = 0; q < S; ++q) lvis[q] |= ((done >> isl(lvis[q])) & 1ull) ? (uint32_t)kNoLevel : 0u;
      wave_lds_sync();
      for (int l = 0; l < dmax; ++l) {
#pragma unroll
        for (int q = 0; q < S; ++q) {  // one slot at a time, busy slots only, as in the velocity passes
          if (lvl(lvis[q]) == l) {
            if constexpr (S > 2) asm volatile("" : "+v"(pw[q]));
            pf2* const pA = reinterpret_cast<pf2*>(s_c + ia(pw[q]));
            pf2* const pB = reinterpret_cast<pf2*>(s_c + ib(pw[q]));
            pf2 cA = *pA, cB = *pB;
            const float sep = solve_position_contact_pk(cA, cB, P.radius, mA, mB);
            *pA = cA;
            *pB = cB;
            // order-preserving int of the float for atomicMin
            const int key = __float_as_int(sep) >= 0 ? __float_as_int(sep) : (__float_as_int(sep) ^ 0x7fffffff);
            atomicMin(&s_pmin[isl(lvis[q])], key);
          }
        }
        wave_lds_sync();
      }
      int km = lane < nisl ? s_pmin[lane] : 0;
      km = km >= 0 ? km : (km ^ 0x7fffffff);
      done |= __builtin_amdgcn_ballot_w64(lane < nisl && !((done >> lane) & 1ull) &&
                                          __int_as_float(km) >= -3.0f * kLinearSlop);
    }
    if (lane < nisl) s_isolved[lane] = (uint8_t)((done >> lane) & 1ull);
  }
};

struct SweepState {
  uint32_t ov_lo, ov_hi;  // partner row of this lane's agent (written by lane j = row owner)
  float best;             // nearest other agent: squared distance
  int bj;                 //                      and index
};

// One record of the all-pairs sweep, unrolled at compile time over J < NCAP (lanes
// >= N hold dummies that overlap nothing and are infinitely far). Each lane shifts its
// overlap bit for agent J into its own partner row (add-with-carry, below); the AABB /
// distance differences run as packed float2 ops, each lane of which is the same IEEE
// operation as the scalar form.
// Records in flight during the sweep: record J + AH is requested while record J is tested,
// so an LDS broadcast has AH records' worth of VALU work to arrive in (a single record's ~12
// VALU do not cover the LDS latency with the other waves of the CU reading too).
constexpr int kSweepAhead = 2;

struct SweepRec {
  float4 fn;
  float2 c;
};

__device__ __forceinline__ SweepRec load_rec(const PairRec* s_pj, int j) {
  SweepRec r;
  r.fn = s_pj[j].fn;  // ds_read_b128
  r.c = s_pj[j].c;    // ds_read_b64 (the pad is never read)
  return r;
}

template <int J, int NCAP, bool NN>
__device__ __forceinline__ void sweep_step(const PairRec* s_pj, SweepRec* win, fvec2 fn_lo, fvec2 fn_hi,
                                           fvec2 cme, unsigned long long valid, int lane, SweepState& st) {
  const SweepRec q = win[J % kSweepAhead];
  if constexpr (J + kSweepAhead < NCAP) win[J % kSweepAhead] = load_rec(s_pj, J + kSweepAhead);
  // b2TestOverlap(fn, fj) separates iff one of (fj.lo - fn.hi, fn.lo - fj.hi) > 0;
  // for finite AABBs (and the +-inf dummies) that is max(...) > 0
  const fvec2 a = mk2(q.fn.x, q.fn.y) - fn_hi;
  const fvec2 b = fn_lo - mk2(q.fn.z, q.fn.w);
  const float sepv = fmaxf(fmaxf(a.x, a.y), fmaxf(b.x, b.y));
  // this lane's overlap bit for agent J (= bit J of its own partner row: the test is
  // symmetric, both orders compare the same four differences) shifted into a per-lane
  // register by add-with-carry (acc = 2 acc + bit): bit J lands at 31 - (J & 31) and is
  // bit-reversed after the sweep; the valid mask is applied there
  (void)valid;
  if constexpr (J < 32)
    asm volatile("v_cmp_nlt_f32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(st.ov_lo) : "v"(sepv) : "vcc");
  else
    asm volatile("v_cmp_nlt_f32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(st.ov_hi) : "v"(sepv) : "vcc");
  if constexpr (NN) {
    const fvec2 d = mk2(q.c.x, q.c.y) - cme;  // other.position - agent.position
    const fvec2 dd = d * d;
    const float d2 = dd.x + dd.y;             // b2DistanceSquared(other, agent)
    // strict '<': lowest index wins ties (mvmnt.py:194); lane J (self) is cleared
    // from the compare mask on the scalar unit. The asm also materialises the
    // running minimum here (otherwise the compiler sinks the distance work past the
    // sweep and spills every record's position).
    asm volatile(
        "v_cmp_lt_f32 vcc, %2, %0\n\t"
        "s_bitset0_b64 vcc, %3\n\t"
        "v_cndmask_b32 %0, %0, %2, vcc\n\t"
        "v_cndmask_b32_e64 %1, %1, %3, vcc"
        : "+v"(st.best), "+v"(st.bj)
        : "v"(d2), "i"(J)
        : "vcc");
    (void)lane;
  }
  // keep the scheduler from hoisting every record's LDS read (register pressure)
  if constexpr ((J & 7) == 7) __builtin_amdgcn_sched_barrier(0);
  if constexpr (J + 1 < NCAP) sweep_step<J + 1, NCAP, NN>(s_pj, win, fn_lo, fn_hi, cme, valid, lane, st);
}

// The sweep's differences as scalar VALU (SCAL) or as v_pk_* pairs: with 16 envs per CU (the
// waves share the SIMDs' issue) the scalar form is 1.9% faster per step, with 4 per CU (1024
// envs: latency-bound) the packed form is 2.2% faster (profiles/r01/ab2 s36). The float32 launch
// with N > 32 picks by the number of envs.
constexpr int kScalarSweepMinEnvs = 2048;

// NCAP = 64 with the nearest neighbour: the records of the two halves are taken in turns
// (0, 32, 1, 33, ...) with a running minimum per half, so the two loop-carried chains (the
// overlap bits of ov_lo / ov_hi and the minimum of each half) are independent and their
// compare -> mask -> select steps issue interleaved; each half's compare result goes to its own
// SGPR pair instead of VCC. Each half still scans its records in increasing j with strict '<',
// and the halves merge with the lower half winning ties, which is the single scan's result.
struct SweepState2 {
  uint32_t ov_lo, ov_hi;
  float best_a, best_b;
  int bj_a, bj_b;
};

template <int S, int AH, bool SCAL>
__device__ __forceinline__ void sweep2_step(const PairRec* s_pj, SweepRec* win, fvec2 fn_lo, fvec2 fn_hi,
                                            fvec2 cme, SweepState2& st) {
  constexpr int JA = S, JB = 32 + S;  // records of this step: JA (lower half), JB (upper half)
  const SweepRec qa = win[(2 * S) % AH], qb = win[(2 * S + 1) % AH];
  // the records of step S + AH / 2 (record order 0, 32, 1, 33, ...)
  if constexpr (2 * S + AH < 64) {
    constexpr int K = 2 * S + AH;
    win[(2 * S) % AH] = load_rec(s_pj, (K & 1) ? 32 + (K >> 1) : (K >> 1));
  }
  if constexpr (2 * S + 1 + AH < 64) {
    constexpr int K = 2 * S + 1 + AH;
    win[(2 * S + 1) % AH] = load_rec(s_pj, (K & 1) ? 32 + (K >> 1) : (K >> 1));
  }
  float sa, sb, d2a, d2b;
  if constexpr (SCAL) {  // see kScalarSweepMinEnvs
  sa = fmaxf(fmaxf(qa.fn.x - fn_hi.x, qa.fn.y - fn_hi.y), fmaxf(fn_lo.x - qa.fn.z, fn_lo.y - qa.fn.w));
  sb = fmaxf(fmaxf(qb.fn.x - fn_hi.x, qb.fn.y - fn_hi.y), fmaxf(fn_lo.x - qb.fn.z, fn_lo.y - qb.fn.w));
  const float dax = qa.c.x - cme.x, day = qa.c.y - cme.y, dbx = qb.c.x - cme.x, dby = qb.c.y - cme.y;
  d2a = dax * dax + day * day;
  d2b = dbx * dbx + dby * dby;
  } else {
  const fvec2 aa = mk2(qa.fn.x, qa.fn.y) - fn_hi, ba = fn_lo - mk2(qa.fn.z, qa.fn.w);
  const fvec2 ab = mk2(qb.fn.x, qb.fn.y) - fn_hi, bb = fn_lo - mk2(qb.fn.z, qb.fn.w);
  sa = fmaxf(fmaxf(aa.x, aa.y), fmaxf(ba.x, ba.y));
  sb = fmaxf(fmaxf(ab.x, ab.y), fmaxf(bb.x, bb.y));
  const fvec2 da = mk2(qa.c.x, qa.c.y) - cme, db = mk2(qb.c.x, qb.c.y) - cme;
  const fvec2 dda = da * da, ddb = db * db;
  d2a = dda.x + dda.y;
  d2b = ddb.x + ddb.y;
  }
  unsigned long long ca, cb, ma, mb;
  asm volatile(
      "v_cmp_nlt_f32_e64 %[ca], 0, %[sa]\n\t"
      "v_cmp_nlt_f32_e64 %[cb], 0, %[sb]\n\t"
      "v_cmp_lt_f32_e64 %[ma], %[da], %[ba]\n\t"
      "v_cmp_lt_f32_e64 %[mb], %[db], %[bb]\n\t"
      "v_addc_co_u32_e64 %[lo], %[ca], %[lo], %[lo], %[ca]\n\t"
      "v_addc_co_u32_e64 %[hi], %[cb], %[hi], %[hi], %[cb]\n\t"
      "s_bitset0_b64 %[ma], %[JA]\n\t"
      "s_bitset0_b64 %[mb], %[JB]\n\t"
      "v_cndmask_b32_e64 %[ba], %[ba], %[da], %[ma]\n\t"
      "v_cndmask_b32_e64 %[ja], %[ja], %[JA], %[ma]\n\t"
      "v_cndmask_b32_e64 %[bb], %[bb], %[db], %[mb]\n\t"
      "v_cndmask_b32_e64 %[jb], %[jb], %[JB], %[mb]"
      : [lo] "+v"(st.ov_lo), [hi] "+v"(st.ov_hi), [ba] "+v"(st.best_a), [bb] "+v"(st.best_b), [ja] "+v"(st.bj_a),
        [jb] "+v"(st.bj_b), [ca] "=&s"(ca), [cb] "=&s"(cb), [ma] "=&s"(ma), [mb] "=&s"(mb)
      : [sa] "v"(sa), [sb] "v"(sb), [da] "v"(d2a), [db] "v"(d2b), [JA] "i"(JA), [JB] "i"(JB));
  if constexpr ((S & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  if constexpr (S + 1 < 32) sweep2_step<S + 1, AH, SCAL>(s_pj, win, fn_lo, fn_hi, cme, st);
}

// New-pair compaction in descending (a, b) order: lane a owns the bitmask of
// partners b > a. Returns the total count; writes at most C entries.
__device__ __forceinline__ int write_new_pairs(int lane, unsigned long long newmask, uint32_t* ocab,
                                               float2* ocimp, int C) {
  const int cnt = __popcll(newmask);
  const int pre = wave_prefix_sum(cnt);  // sum over lanes <= lane
  const int total = __builtin_amdgcn_readlane(pre, W - 1);
  int w = total - pre;  // the lanes above this one: they write first (descending a)
  unsigned long long m = newmask;
  while (m) {
    const int j = 63 - __clzll(m);
    m &= ~(1ull << j);
    if (w < C) {
      st_g<kState>(ocab + w, (uint32_t)lane | ((uint32_t)j << 16));
      st_g<kState>(ocimp + w, make_float2(0.0f, 0.0f));
    }
    ++w;
  }
  return total;
}

// ---- the tail observation (round 6) -----------------------------------------------------------------
// A TDM trajectory rollout whose envs all fit the chip at once. The fused form observes inside each
// env's wave after every step (55% of a wave's cycles at 2 x 16), so the launch ends with the heaviest
// env's K physics steps plus its K observations. Here every wave steps its env's K steps writing
// only pose snapshots (write-through, st_wt4) and, each step, the number of its steps whose snapshots
// have drained (its ready word); a wave that has finished its own steps then observes (step, env) rows
// in step-major order from a shared counter, each once its env's ready word covers the step, until
// all K x E rows are taken. Extra blocks (blockIdx.x >= E) only observe. The observations of the envs
// that end first run beside the heaviest envs' physics. A wait that does not end within ~1 s (never
// expected: every env's wave is resident, macm_capi checks the occupancy, and never waits) reports
// MACM_ST_HANDOFF and ends the worker. Each row is the fused form's observation of the same snapshot
// values (tdm_obs_rowblocks / tdm_obs_pairs), bit for bit.
struct TailObs {
  unsigned long long* ctl;  // tail_ctl_words(E) words (flock_common.hpp): row counters, then ready words
  unsigned int tag;         // this launch's tag (> 0); the ready word of env e holds tag << 32 | steps stored
  int nsteps;               // the steps observed in the tail: the launch's last nsteps (k0 = K - nsteps)
  int k;                    // physics: the tail step this call takes (tail steps 0 .. k - 1 are complete;
                            // negative: a step before the tail, observed in the step itself)
  bool worker;              // this call observes one claimed row instead of stepping
  bool more;                // worker: false once every row is taken (or a wait gave up)
  int q, left;              // worker: the sub-queue it claims from, sub-queues not yet found empty
  int r, r_end;             // worker: the rows of its current claim (sub-queue-local, step-major)
  int nq;                   // sub-queues in use: min(kTailQ, blocks of the launch), each with a wave
};
// The rows are split into kTailQ sub-queues by env range (a single counter, one device-scope atomic
// per row, serialised at ~9 ns per claim: 81,920 rows of C4 cost more than the observation saved); a
// worker takes kTailChunk rows per claim from sub-queue blockIdx % kTailQ only and ends when it is
// empty (moving on to the other sub-queues cost every leaving wave kTailQ accesses to the same few
// lines: ~5 us per step at 4096 envs).
constexpr int kTailChunk = 2;
constexpr unsigned kTailSpins = 1u << 20;

__device__ __forceinline__ unsigned long long* tail_counter(const TailObs& tl, int q) {
  return tl.ctl + (size_t)(((tl.tag & 1u) * kTailQ + q) * kTailLine);
}

template <typename OT>
__device__ __forceinline__ void tdm_tail_row(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                                             const TdmBuffers& TB, OT* obs, TailObs& tl, int lane, float2* s_c,
                                             float* s_ang, float4* stage, bool staged) {
  const int E = P.n_envs, N = P.n_agents;
  const int nq = tl.nq > 0 ? tl.nq : 1;
  auto env0 = [E, nq](int q) { return (int)(((long long)E * q) / nq); };
  while (tl.r >= tl.r_end) {  // claim kTailChunk rows of the current sub-queue, else move on
    if (tl.left == 0) {
      tl.more = false;
      return;
    }
    const int ne = env0(tl.q + 1) - env0(tl.q);
    const int nrows = tl.nsteps * ne;
    int c = 0;
    if (lane == 0 && ne > 0) {
      // a load first: the waves leaving find every sub-queue empty, and a load of an exhausted counter
      // does not queue behind the other waves' atomics on it
      unsigned long long* const ctr = tail_counter(tl, tl.q);
      const unsigned long long seen = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      c = seen * kTailChunk >= (unsigned long long)nrows
              ? (int)seen
              : (int)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    c = __builtin_amdgcn_readfirstlane(c);
    if (ne == 0 || (long long)c * kTailChunk >= nrows) {
      tl.q = tl.q + 1 == nq ? 0 : tl.q + 1;
      --tl.left;
      continue;
    }
    tl.r = c * kTailChunk;
    tl.r_end = min(tl.r + kTailChunk, nrows);
  }
  const int e0 = env0(tl.q), ne = env0(tl.q + 1) - e0;
  const int i = tl.r++;
  const int k = i / ne, e = e0 + (i - k * ne);
  if (k >= tl.nsteps || e >= E || e < 0) {  // never: a row outside the launch ends the worker, not a fault
    if (lane == 0) report_status(B, MACM_ST_HANDOFF);
    tl.more = false;
    return;
  }
  int ok = 1;
  if (lane == 0) {
    ok = 0;
    for (unsigned it = 0; it < kTailSpins; ++it) {
      const unsigned long long v = __hip_atomic_load(tl.ctl + 2 * kTailQ * kTailLine + e, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
      if ((unsigned)(v >> 32) == tl.tag && (unsigned)v > (unsigned)k) {
        ok = 1;
        break;
      }
      if (it < 16) __builtin_amdgcn_s_sleep(2);
      else __builtin_amdgcn_s_sleep(32);  // a long wait: poll ~1 us apart
    }
    if (!ok) report_status(B, MACM_ST_HANDOFF);
  }
  if (!__builtin_amdgcn_readfirstlane(ok)) {
    tl.more = false;
    return;
  }
  const size_t srow = ((size_t)k * E + e) * N;  // the snapshot row: [nsteps, E, N]
  float4 sn = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (lane < N) sn = ld_wt4(TB.snap_out + srow + lane);
  const size_t row = ((size_t)(tl.k + k) * E + e) * N;  // the observation row of launch step k0 + k (tl.k: k0)
  s_c[lane] = make_float2(sn.x, sn.y);
  s_ang[lane] = sn.z;
  const unsigned long long livem = __ballot(lane < N && sn.w != 0.0f);
  __syncthreads();
  const size_t slots = row * (N - 1);
  OT* const obs_r = obs ? obs + slots * 4 : nullptr;
  uint8_t* const mask_r = TB.mask_out ? TB.mask_out + slots : nullptr;
  if constexpr (sizeof(OT) == 4) {
    if (staged) tdm_obs_rowblocks<OT>(obs_r, mask_r, N, lane, livem, TP, s_c, s_ang, stage, true);
    else tdm_obs_pairs<OT>(obs_r, mask_r, N, lane, livem, TP, s_c, s_ang);
  } else {
    tdm_obs_pairs<OT>(obs_r, mask_r, N, lane, livem, TP, s_c, s_ang);
  }
  __syncthreads();  // the next row's snapshot overwrites s_c, s_ang and the stage
}

// MODE kFlock: Flock.step. MODE kTdm: TDM.step (combat.py:104-184) — the same
// physics with alive masks, plus melee ray casts, health, deaths and the full
// relative observation; `TP`/`TB` are unused for Flock.
// waves_per_eu(4): <= 128 VGPRs, so the 16 envs per CU of a 4096-env launch are
// resident together (the unrolled sweep would otherwise hoist every LDS record).
// The body of one step of env blockIdx.x, inlined into the one-step kernel (env_step_w64) and
// the multi-step kernel (env_rollout_w64); its LDS arrays are the kernel's.
template <int MODE, int NCAP, typename OT, bool SCAL = false>
__device__ __attribute__((always_inline)) inline void step_w64_body(
    const StepParams& P, const WorldBuffers& B, const TdmParams& TP, const TdmBuffers& TB, int cur,
    const void* __restrict__ actions, OT* __restrict__ obs, int32_t* __restrict__ nbr_out,
    float* __restrict__ rew_out, uint8_t* __restrict__ coll_out, uint8_t* __restrict__ done_out,
    const int e = blockIdx.x, const int lane = threadIdx.x, TailObs* tl = nullptr) {
  constexpr bool kT = MODE == kTdm;
#ifdef MACM_TIMELINE
  const unsigned long long tl_rt0 = __builtin_amdgcn_s_memrealtime(), tl_c0 = __builtin_amdgcn_s_memtime();
#endif
  const int N = P.n_agents;
  const int C = P.max_contacts;
  // a body that takes part in the physics: every agent (Flock) / alive agents (TDM;
  // body.active = False removes the proxy and its contacts, combat.py:162)
  bool act = lane < N;
  const size_t ag = (size_t)e * N + lane;
  const int nxt = cur ^ 1;
  const unsigned long long lt = lanemask_lt(lane);

  __shared__ float2 s_c[W];  // positions (one 8-byte access per body)
  __shared__ float2 s_v[W];  // velocities (one ds_read_b64 / ds_write_b64 per body)
  // per agent: bit mask of its touching contacts for the scalar DFS (T <= 64 TMW); TDM keeps one
  // 64-bit word (its LDS budget is full), Flock two
  constexpr int TMW = kT ? 1 : 2;
  // The contact arrays in one block, which the spill step (flock_spill.hpp) reuses as its
  // per-body LDS when an env's touching contacts overflow TCAP / DEG.
  struct __align__(32) Pool {
    // contact normals live until the velocity solve ends and the pairs until the position
    // solve ends; the all-pairs records are written after it over both
    float tn[2 * TCAP];
    uint32_t tab[TCAP];
    float tln[TCAP], tlt[TCAP];
    uint32_t tm[2 * TMW * W];
    uint32_t oldm[2 * W];  // per agent: 64-bit mask of partners in the old list
  };
  __shared__ Pool s_pool;
  static_assert(spill::layout(W, !kT).total <= (int)sizeof(Pool), "the spill step must fit the pool");
  uint32_t* const s_tab = s_pool.tab;
  float* const s_tln = s_pool.tln;
  float* const s_tlt = s_pool.tlt;
  float* const s_tn = s_pool.tn;
  float* const s_tnx = s_tn;
  float* const s_tny = s_tn + TCAP;
  PairRec* const s_pj = reinterpret_cast<PairRec*>(s_tn);
  // s_pj spans s_tn and s_tab (adjacent in Pool): both are dead once the position solve ends
  static_assert(offsetof(Pool, tab) == sizeof(float) * 2 * TCAP, "tab must follow tn");
  static_assert(sizeof(PairRec) * W <= sizeof(float) * 2 * TCAP + sizeof(uint32_t) * TCAP, "s_pj must fit in s_tn + s_tab");
  uint32_t* const s_tm = s_pool.tm;
  uint32_t* const s_oldm = s_pool.oldm;
  // per-body touching edges when T > 64 TMW (no scalar DFS); Flock: in s_tm's words, which only
  // the scalar DFS reads
  __shared__ uint8_t s_adj_tdm[kT ? W * DEG : 1];
  uint8_t* const s_adj = kT ? s_adj_tdm : reinterpret_cast<uint8_t*>(s_pool.tm);
  static_assert(kT || sizeof(uint32_t) * 2 * 2 * W >= W * DEG, "s_adj must fit in s_tm");
  static_assert(sizeof(uint32_t) * 2 * TMW * W >= sizeof(float2) * W, "the level steps' dummy slots must fit in s_tm");
  __shared__ uint8_t s_ord[TCAP];
  __shared__ uint32_t s_cvis[TCAP / 32];
  __shared__ uint8_t s_deg[W], s_stack[W], s_ibodies[W], s_bisl[W];
  __shared__ uint16_t s_ic[ICAP + 1];
  __shared__ uint8_t s_ib[ICAP + 1];
  __shared__ uint8_t s_isolved[ICAP];
  __shared__ uint32_t s_imin[ICAP];  // per island: min sleep time (float bits, all >= 0)
  __shared__ int s_nisl;
  // TDM only (unreferenced, hence not allocated, in the Flock instantiation)
  __shared__ double s_hpd[W];
  __shared__ int8_t s_hit[W];
  __shared__ float s_ang[W];
#ifdef MACM_STAMPS
  __shared__ int s_stat_maxisl;
#endif
  if constexpr (kT) {
    if (tl && tl->worker) {  // the tail observation: one (step, env) row instead of a step
      tdm_tail_row<OT>(P, B, TP, TB, obs, *tl, lane, s_c, s_ang, reinterpret_cast<float4*>(&s_pool),
                       tdm_obs_rb_stage_bytes(N) <= (int)sizeof(Pool));
      return;
    }
  }

  // ---- every global load the step needs, issued up front ---------------------
  const uint32_t* cab = B.cab[cur] + (size_t)e * C;
  const float2* cimp = B.cimp[cur] + (size_t)e * C;
  const int step_count = B.step_count[e];
  const int M = B.ccount[cur][e];
  float2 p = make_float2(0.0f, 0.0f), v = make_float2(0.0f, 0.0f), tg = make_float2(0.0f, 0.0f);
  float ang = 0.0f, slp = 0.0f;
  float4 fo = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  int a0 = 1, a1 = 1, a2 = 1, a3 = 0;
  float ax = 0.0f, ay = 0.0f;
  double hp = 0.0, cda = 0.0, cdm = 0.0;  // TDM: health, cooldown_atk, cooldown_mov_penalty
  if (act) {
    p = B.pos[ag];
    v = B.vel[ag];
    ang = B.angle[ag];
    fo = B.fat[ag];
    slp = B.sleep[ag];
    if constexpr (kT) {
      const uchar4 a = reinterpret_cast<const uchar4*>(actions)[ag];
      a0 = a.x;
      a1 = a.y;
      a2 = a.z;
      a3 = a.w;
      act = TB.alive[ag] != 0;
      hp = TB.health[ag];
      cda = TB.cd_atk[ag];
      cdm = TB.cd_mov[ag];
    } else if (P.action_mode == MACM_ACTION_DISCRETE) {
      const uint8_t* a = (const uint8_t*)actions + ag * 3;
      a0 = a[0];
      a1 = a[1];
      a2 = a[2];
    } else {
      const float2 c = ((const float2*)actions)[ag];
      ax = c.x;
      ay = c.y;
    }
    if constexpr (!kT) tg = B.targets[(size_t)e * P.n_targets + B.tidx[lane]];
  }
  const bool act0 = act;  // TDM: alive when the step starts (acts this step)
  double time_passed = 0.0;
  int st_prev = 0;
  unsigned long long ctr[4] = {0ull, 0ull, 0ull, 0ull};
  int2 lis = make_int2(0, -1);
  int win_prev = -1;
  uint8_t done_prev = 0;
  if (lane == 0) {
    time_passed = B.time_passed[e];
    st_prev = B.status[e];
    if constexpr (kT) {
      lis = TB.listener[e];
      win_prev = TB.winner[e];
      done_prev = B.done[e];
    }
    const ulonglong2* ec = reinterpret_cast<const ulonglong2*>(B.env_counters + (size_t)e * 4);
    const ulonglong2 c01 = ec[0], c23 = ec[1];
    ctr[0] = c01.x;
    ctr[1] = c01.y;
    ctr[2] = c23.x;
    ctr[3] = c23.y;
  }
  // list entries (and their warm-start impulses) of the first RCH chunks stay in registers
  uint32_t rab[RCH];
  float2 rim[RCH];
#pragma unroll
  for (int c = 0; c < RCH; ++c) {
    const int k = c * W + lane;
    rab[c] = 0u;
    rim[c] = make_float2(0.0f, 0.0f);
    if (k < M) {
      rab[c] = cab[k];
      rim[c] = cimp[k];
    }
  }
  s_c[lane] = p;
  if (lane < TCAP / 32) s_cvis[lane] = 0u;
  s_oldm[2 * lane] = 0u;
#pragma unroll
  for (int q = 0; q < 2 * TMW; ++q) s_tm[2 * TMW * lane + q] = 0u;
  s_oldm[2 * lane + 1] = 0u;
  int status = 0;
  STAMP(0);

  // ---- actions -> angle, force (mvmnt.py:97-129, combat.py:121-139) ----------
  float Fx = 0.0f, Fy = 0.0f;
  bool attacking = false;
  float ray_x = 0.0f, ray_y = 0.0f;
  if (act) {
    if (P.action_mode == MACM_ACTION_DISCRETE) {
      // agent.body.angle = angle + (a2-1) * rotation_speed * (1/hz) -> SetTransform(float32)
      float af = (float)((double)ang + ((double)(a2 - 1) * P.rot_step) * P.inv_hz);
      double ad = (double)af;
      if (fabs(ad) > M_PI) {
        af = (float)(ad - sgn(ad) * (2.0 * M_PI));
        ad = (double)af;
      }
      ang = af;
      const double cc = ((a0 != 1) && (a1 != 1)) ? P.diag_c : 1.0;
      const double k0 = (double)(a0 - 1), k1 = (double)(a1 - 1);
      double force = P.force;
      // Agent.force = _force * (1 - percent_mov_penalty * int(cooldown_mov_penalty > 0))   combat.py:46-49
      if constexpr (kT) force = P.force * (1.0 - TP.percent_mov_penalty * (double)(cdm > 0.0));
      double s0, c0, s1, c1;  // np.cos / np.sin of angle and angle + pi/2 (one reduction each)
      act_trig(af, &s0, &c0, &s1, &c1);
      const double fx = (c0 * k0 + c1 * k1) * cc * force;
      const double fy = (s0 * k0 + s1 * k1) * cc * force;
      Fx = (float)fx;  // ApplyForce: b2Vec2(float32) accumulated onto m_force = 0
      Fy = (float)fy;
      if constexpr (kT) {  // melee (combat.py:141-155)
        if (cda <= 0.0) {
          if (a3) {
            attacking = true;
            // point2 = point1 + (range*cos(angle), range*sin(angle)): b2Vec2 + tuple is a
            // float32 add of the float32-converted tuple
            ray_x = p.x + (float)(TP.melee_range * c0);  // c0 = cos(angle), s0 = sin(angle)
            ray_y = p.y + (float)(TP.melee_range * s0);
            cda = TP.cooldown_atk;
            cdm = TP.cooldown_mov_penalty;
          }
        } else {
          cda -= P.inv_hz;
          if (TP.decay_mov_penalty) cdm -= P.inv_hz;
        }
      }
    } else {
      float x = ax, y = ay;
      if ((x * x + y * y) > 1.0f) {
        x = sqrtf(x * x / (x * x + y * y));
        y = sqrtf(y * y / (x * x + y * y));
      }
      Fx = x * P.force_f32;
      Fy = y * P.force_f32;
    }
    Fx = 0.0f + Fx;  // m_force += force, from ClearForces' zero
    Fy = 0.0f + Fy;
  }
  unsigned long long att_m = 0ull, alive0_m = 0ull;
  if constexpr (kT) {
    // Ray casts. Bodies do not move during the action loop (SetTransform keeps the
    // position) and deaths come after it, so every cast sees the same world: all
    // rays are cast in parallel; only the listener update is ordered.
    alive0_m = __ballot(act);
    att_m = __ballot(attacking);
    s_hpd[lane] = hp;
    __syncthreads();  // s_c / s_hpd visible
    if (att_m) {
      // b2World::RayCast + RayCastClosestCallback (cm_framework.py:56-86): each
      // b2CircleShape::RayCast hit clips maxFraction to its fraction; candidates in
      // body order, as the oracle (b2l_world_raycast)
      int hit = -1;
      const float rvx = ray_x - p.x, rvy = ray_y - p.y;  // r = p2 - p1
      const float rrr = rvx * rvx + rvy * rvy;
      const float rad2 = P.radius * P.radius;
      float maxf = 1.0f;
      for (unsigned long long m = alive0_m; m; m &= m - 1ull) {
        const int j = __builtin_ctzll(m);
        const float2 cj = s_c[j];
        const float sx = p.x - cj.x, sy = p.y - cj.y;  // s = p1 - position
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
      s_hit[lane] = (int8_t)(attacking ? hit : -1);
      __syncthreads();
      if (lane == 0) {
        // listener.hit / listener.fixture persist across casts and steps (literal), or
        // reset per cast (fresh_raycast); damage in agent order (combat.py:152-153)
        for (unsigned long long m = att_m; m; m &= m - 1ull) {
          const int h = s_hit[__builtin_ctzll(m)];
          if (TP.fresh_raycast) {
            if (h >= 0) s_hpd[h] -= TP.melee_dmg;
          } else {
            if (h >= 0) lis = make_int2(1, h);
            if (lis.x) s_hpd[lis.y] -= TP.melee_dmg;
          }
        }
      }
      __syncthreads();
      hp = s_hpd[lane];
    }
    if (act && hp <= 0.0) act = false;  // deaths: body.active = False (combat.py:157-165)
  }
  // bodies in the physics step (Flock: all N; TDM: alive after this step's deaths)
  const unsigned long long livem = __ballot(act);
  __syncthreads();
  STAMP(1);

  // ---- Collide: touching contacts of the ordered list ---------------------
  const float rr = (P.radius + P.radius) * (P.radius + P.radius);
  const float dt_ratio = step_count > 0 ? P.inv_dt * P.dt : 0.0f;  // m_inv_dt0 * dt
  int T = 0;
  uint32_t tbits = 0u;  // bit c: this lane's entry of chunk c touches (M <= C <= 2016 -> < 32 chunks)
  for (int c = 0; c * W < M; ++c) {
    const int k = c * W + lane;
    uint32_t ab = 0u;
    float2 lam = make_float2(0.0f, 0.0f);
    if (c < RCH) {
#pragma unroll
      for (int q = 0; q < RCH; ++q)
        if (q == c) {
          ab = rab[q];
          lam = rim[q];
        }
    } else if (k < M) {
      ab = cab[k];
      lam = cimp[k];
    }
    bool touch = false;
    float tnx = 1.0f, tny = 0.0f;
    if (k < M) {
      const int a = ab & 0xffffu, b = ab >> 16;
      // TDM: contacts of a body that died this step were destroyed with its proxy
      if (!kT || ((livem >> a) & (livem >> b) & 1ull)) {
        const float2 ca = s_c[a], cb = s_c[b];
        const float dx = cb.x - ca.x, dy = cb.y - ca.y;
        touch = !(dx * dx + dy * dy > rr);  // b2CollideCircles
        if (touch) {
          // the contact normal from the same start-of-step positions (InitializeVelocityConstraints:
          // (1, 0) when the centres coincide; (pA - pB)^2 == (pB - pA)^2 exactly)
          if (dx * dx + dy * dy > kEps * kEps) {
            tnx = dx;
            tny = dy;
            normalize(tnx, tny);
          }
        }
        atomicOr(&s_oldm[2 * a + (b >> 5)], 1u << (b & 31));
        atomicOr(&s_oldm[2 * b + (a >> 5)], 1u << (a & 31));
      }
    }
    const unsigned long long m = __ballot(touch);
    if (touch) {
      tbits |= 1u << c;
      const int slot = T + __popcll(m & lt);
      if (slot < 64 * TMW) {  // touching contact `slot` of both bodies (the scalar DFS below)
        atomicOr(&s_tm[2 * TMW * (ab & 0xffffu) + (slot >> 5)], 1u << (slot & 31));
        atomicOr(&s_tm[2 * TMW * (ab >> 16) + (slot >> 5)], 1u << (slot & 31));
      }
      if (slot < TCAP) {
        s_tab[slot] = ab;
        s_tln[slot] = P.warm_starting ? dt_ratio * lam.x : 0.0f;
        s_tlt[slot] = P.warm_starting ? dt_ratio * lam.y : 0.0f;
        s_tnx[slot] = tnx;
        s_tny[slot] = tny;
      }
    }
    T += __popcll(m);
  }
  const bool touch_over = T > TCAP;
  if (touch_over) {
    status |= MACM_ST_TOUCH_OVERFLOW;
    T = TCAP;
  }
  __syncthreads();
  STAMP(2);

  // ---- per-body touching edges in list (= Box2D edge) order ----------------
  // T <= 64 TMW (the common case): a body's edges are the set bits of its touching mask, in
  // ascending contact order = list order. Otherwise an explicit edge array per body.
  const bool fast_dfs = T <= 64 * TMW;
  int deg = 0;
  unsigned long long tmask = 0ull, tmask1 = 0ull;  // contacts 0..63, 64..127
  if (fast_dfs) {
    if (act) {
      const uint32_t* tm = s_tm + 2 * TMW * lane;
      tmask = (unsigned long long)tm[0] | ((unsigned long long)tm[1] << 32);
      if (TMW == 2 && T > 64) tmask1 = (unsigned long long)tm[2] | ((unsigned long long)tm[3] << 32);
      deg = __popcll(tmask) + __popcll(tmask1);
    }
  } else if (act) {
    for (int t = 0; t < T; ++t) {
      const uint32_t ab = s_tab[t];
      if ((int)(ab & 0xffffu) == lane || (int)(ab >> 16) == lane) {
        if (deg < DEG) s_adj[lane * DEG + deg] = (uint8_t)t;
        ++deg;
      }
    }
  }
  if constexpr (!kT) {
    // More touching contacts than TCAP, or a body with more than DEG: the env is stepped by the
    // spill step instead (HBM working set, flock_spill.hpp). Nothing has been written to global
    // memory yet, so it starts from the untouched start-of-step state; this wave returns after it.
    // (The scalar DFS of T <= 64 TMW has no degree cap: it walks bit masks.)
    if (touch_over || (!fast_dfs && __builtin_amdgcn_ballot_w64(deg > DEG) != 0ull) || P.force_spill) {
      spill::step_env<OT, true>(P, B, e, cur, actions, obs, nbr_out, rew_out, coll_out, done_out,
                                reinterpret_cast<unsigned char*>(&s_pool));
      return;
    }
  } else {
    // TDM: the same hand-over, after this step's actions, casts and deaths; the spill step does the
    // physics of the living bodies and TDM's env layer (its records in HBM: the pool is smaller)
    if (touch_over || (!fast_dfs && __builtin_amdgcn_ballot_w64(deg > DEG) != 0ull) || P.force_spill) {
      // The spill working-set slot is taken before anything of this step is committed: a pool that
      // stays full (~1 s) leaves the env wholly unstepped and reported, never half-stepped (ADVICE
      // r03, as the workgroup TDM step does)
      __shared__ int s_slot;
      const int slot = spill::acquire_slot(B, e, &s_slot);
      if (slot < 0) {
        spill::keep_lists(P, B, e, cur);
        if (lane == 0) {
          B.status[e] |= MACM_ST_SPILL_WAIT;
          report_status(B, MACM_ST_SPILL_WAIT);
        }
        return;
      }
      // the combat state of this step is committed first (the spill step reads it back: nothing
      // of it stays live in registers across the spill step)
      if (lane < N) {
        if (act0) {
          B.angle[ag] = ang;
          TB.cd_atk[ag] = cda;
          TB.cd_mov[ag] = cdm;
        }
        TB.health[ag] = hp;
        TB.alive[ag] = act ? 1 : 0;
        if (TB.health_out) TB.health_out[ag] = hp;
        if (TB.alive_out) TB.alive_out[ag] = act ? 1 : 0;
      }
      if (lane == 0) {
        TB.listener[e] = lis;
        ulonglong2* ec = reinterpret_cast<ulonglong2*>(B.env_counters + (size_t)e * 4);
        ec[0] = make_ulonglong2(ctr[0] + (unsigned long long)__popcll(alive0_m),
                                ctr[1] + (unsigned long long)__popcll(att_m));
        B.env_counters[(size_t)e * 4 + 2] = ctr[2] + (unsigned long long)__popcll(alive0_m & ~livem);
      }
      const float2 F1 = make_float2(Fx, Fy);
      spill::step_env<OT, false, kTdm>(P, B, e, cur, actions, obs, nullptr, nullptr, nullptr, done_out,
                                        reinterpret_cast<unsigned char*>(&s_pool), &TP, &TB, &F1, slot);
      return;
    }
  }
  if (!fast_dfs && deg > DEG) {
    status |= MACM_ST_DEGREE_OVERFLOW;
    deg = DEG;
  }
  if (!fast_dfs) s_deg[lane] = (uint8_t)deg;
  const unsigned long long hasdeg = __ballot(act && deg > 0);
  __syncthreads();
  STAMP(3);
  // The serial Box2D chain (DFS, Gauss-Seidel, position passes) is a latency chain; the
  // waves sharing this SIMD run throughput phases (sweep, obs) that can fill its gaps.
  // Raising the issue priority of a wave that has touching contacts while it walks the
  // chain (3), and keeping it above the contact-free waves afterwards (1 or 2, below), shortens the
  // envs with the most contacts, which set the kernel's duration (tools/timeline.py:
  // waves end at 15.5 us median, 25 us at the latest). Measured -8% per step at the metric
  // config against no priority; per-island-size or list-size priorities did no better.
  if (hasdeg) __builtin_amdgcn_s_setprio(3);

  // ---- island DFS in Box2D order (b2World::Solve), serial on lane 0 --------
  // Seeds in body-list order (reverse creation); bodies without touching
  // edges are singleton islands and contribute no contact order, so only
  // bodies in `hasdeg` are walked.
  uint32_t ordv = 0u, lvlv = 0u, kislv = 0u;  // lane k: the k-th contact in island order, its level, island
  bool lvl_path = fast_dfs && T <= 64;  // narrowed after the DFS (largest island)
  if (fast_dfs) {
    // Wave-uniform (scalar) DFS: bodies' edge masks and contacts' pairs are read from the
    // owning lanes' registers (v_readlane), visited sets are 64-bit masks, and the outputs
    // and the stack are built in registers lane by lane (v_writelane), so the walk touches
    // no LDS. Visiting all unvisited edges of a popped body in ascending order is Box2D's
    // edge walk (an edge is only ever marked by its own visit).
    const uint32_t tabv = lane < T ? s_tab[lane] : 0u;  // contact `lane`'s pair
    const uint32_t tabv1 = (TMW == 2 && 64 + lane < T) ? s_tab[64 + lane] : 0u;  // contact 64 + lane's
    const uint32_t tm_lo = (uint32_t)tmask, tm_hi = (uint32_t)(tmask >> 32);
    const uint32_t tm1_lo = (uint32_t)tmask1, tm1_hi = (uint32_t)(tmask1 >> 32);
    uint32_t ordv1 = 0u, bodv = 0u, islv = 0u, icv = 0u, ibv = 0u, stk = 0u;
    int nord = 0, nisl = 0, nb = 0;
    // one instantiation per width so that the common T <= 64 walk carries no second word
    auto dfs = [&](auto wide) {
    constexpr bool W2 = decltype(wide)::value;
    unsigned long long vis = ~hasdeg, cvis = 0ull, cvis1 = 0ull;
    for (unsigned long long todo = hasdeg; todo; todo = hasdeg & ~vis) {
      const int s = 63 - __clzll(todo);
      icv = writelane_m0(nord, nisl, icv);  // s_ic[nisl]
      ibv = writelane_m0(nb, nisl, ibv);    // s_ib[nisl]
      vis |= 1ull << s;
      stk = writelane_m0(s, 0, stk);
      int sp = 1;
      while (sp > 0) {
        --sp;
        const int b = __builtin_amdgcn_readlane(stk, sp);
        bodv = writelane_m0(b, nb, bodv);  // s_ibodies[nb]
        islv = writelane_m0(nisl, b, islv);  // s_bisl[b]
        ++nb;
        // the body's unvisited edges in ascending contact order: contacts 0..63, then 64..127
        auto walk = [&](unsigned long long m, int base, uint32_t tab) {
          while (m) {
            const int t = __builtin_ctzll(m);
            m &= m - 1ull;
            // s_ord[nord]: lane nord % 64 of ordv; the first 64 entries are set aside in ordv1 once
            // complete (a select, instead of a branch between two registers on every edge)
            ordv = writelane_m0(base + t, W2 ? (nord & 63) : nord, ordv);
            const uint32_t ab = (uint32_t)__builtin_amdgcn_readlane(tab, t);
            const int a = ab & 0xffffu, bb = ab >> 16;
            ++nord;
            if constexpr (W2) ordv1 = nord == 64 ? ordv : ordv1;
            const int o = (a == b) ? bb : a;
            if ((vis >> o) & 1ull) continue;
            vis |= 1ull << o;
            stk = writelane_m0(o, sp, stk);
            ++sp;
          }
        };
        unsigned long long m = (((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(tm_hi, b) << 32) |
                                (unsigned long long)(uint32_t)__builtin_amdgcn_readlane(tm_lo, b)) & ~cvis;
        cvis |= m;
        walk(m, 0, tabv);
        if constexpr (W2) {
          unsigned long long m1 = (((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(tm1_hi, b) << 32) |
                                   (unsigned long long)(uint32_t)__builtin_amdgcn_readlane(tm1_lo, b)) & ~cvis1;
          cvis1 |= m1;
          walk(m1, 64, tabv1);
        }
      }
      ++nisl;
    }
    };
    if (TMW == 2 && T > 64) dfs(BoolC<true>{});
    else dfs(BoolC<false>{});
    icv = writelane_m0(nord, nisl, icv);
    ibv = writelane_m0(nb, nisl, ibv);
    const bool wrapped = TMW == 2 && nord > 64;  // entries 0..63 in ordv1, 64.. in ordv
    if (lane < nord) s_ord[lane] = (uint8_t)(wrapped ? ordv1 : ordv);
    if (TMW == 2 && 64 + lane < nord) s_ord[64 + lane] = (uint8_t)ordv;
    if (lane < nb) s_ibodies[lane] = (uint8_t)bodv;
    if ((hasdeg >> lane) & 1ull) s_bisl[lane] = (uint8_t)islv;
    if (lane <= nisl) {
      s_ic[lane] = (uint16_t)icv;
      s_ib[lane] = (uint8_t)ibv;
    }
    if (lane == 0) {
      s_nisl = nisl;
#ifdef MACM_STAMPS
      int mx = 0;
      for (int q = 0; q < nisl; ++q) mx = max(mx, __builtin_amdgcn_readlane(icv, q + 1) - __builtin_amdgcn_readlane(icv, q));
      s_stat_maxisl = mx;
#endif
    }
  }
  if (!fast_dfs && lane == 0 && hasdeg) {
    unsigned long long vis = ~hasdeg;
    int nord = 0, nisl = 0, nb = 0;
    for (unsigned long long todo = hasdeg; todo; todo = hasdeg & ~vis) {
      const int s = 63 - __clzll(todo);
      s_ic[nisl] = (uint16_t)nord;
      s_ib[nisl] = (uint8_t)nb;
      int sp = 0;
      s_stack[sp++] = (uint8_t)s;
      vis |= 1ull << s;
      while (sp > 0) {
        const int b = s_stack[--sp];
        s_bisl[b] = (uint8_t)nisl;
        s_ibodies[nb++] = (uint8_t)b;
        const int db = s_deg[b];
        for (int q = 0; q < db; ++q) {
          const int t = s_adj[b * DEG + q];
          const uint32_t bit = 1u << (t & 31);
          if (s_cvis[t >> 5] & bit) continue;
          s_cvis[t >> 5] |= bit;
          s_ord[nord++] = (uint8_t)t;
          const uint32_t ab = s_tab[t];
          const int a = ab & 0xffffu, bb = ab >> 16;
          const int o = (a == b) ? bb : a;
          if ((vis >> o) & 1ull) continue;
          vis |= 1ull << o;
          s_stack[sp++] = (uint8_t)o;
        }
      }
      ++nisl;
    }
    s_ic[nisl] = (uint16_t)nord;
    s_ib[nisl] = (uint8_t)nb;
    s_nisl = nisl;
#ifdef MACM_STAMPS
    {
      int mx = 0;
      for (int q = 0; q < nisl; ++q) mx = max(mx, (int)s_ic[q + 1] - (int)s_ic[q]);
      s_stat_maxisl = mx;
    }
#endif
  }
  if (!fast_dfs && lane == 0 && !hasdeg) {
    s_nisl = 0;
#ifdef MACM_STAMPS
    s_stat_maxisl = 0;
#endif
  }

  // ---- integrate velocities + damping (b2Island::Solve) --------------------
  float vx = v.x, vy = v.y;
  if (act) {
    vx = vx + P.dt * (0.0f + P.inv_mass * Fx);  // gravityScale * gravity == 0
    vy = vy + P.dt * (0.0f + P.inv_mass * Fy);
    vx = vx * P.damp;
    vy = vy * P.damp;
  }
  s_v[lane] = make_float2(vx, vy);

  __syncthreads();
  STAMP(4);
  if constexpr (kT) {
    // the tail observation: steps 0 .. k - 1 are complete and their write-through snapshot stores
    // drained by now (waiting here costs nothing: this step has stored nothing yet), so the ready word
    // can say k
    if (tl && tl->ctl && tl->k > 0) {
      __builtin_amdgcn_s_waitcnt(0);
      if (lane == 0)
        __hip_atomic_store(tl->ctl + 2 * kTailQ * kTailLine + e, ((unsigned long long)tl->tag << 32) | (unsigned)tl->k,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  const int nisl = s_nisl;
  const float mA = P.inv_mass, mB = P.inv_mass;
  const float kmass = (mA + mB) > 0.0f ? 1.0f / (mA + mB) : 0.0f;  // normalMass == tangentMass
  const float friction = P.friction;

  // ---- warm start + velocity iterations, one lane per island ---------------
  // A single-contact island (the common case) runs entirely in registers; larger
  // islands go through LDS in Box2D's order.
  // any 2..KREC-contact island in this wave (wave-uniform; nisl <= ICAP < W, one island per lane)
  const int lsz = lane < nisl ? s_ic[lane + 1] - s_ic[lane] : 0;
  const bool krec_wave = __builtin_amdgcn_ballot_w64(lsz >= 2 && lsz <= KREC) != 0ull;
  // levels pay off once an island is longer than the register-record path takes (KREC): islands
  // of up to KREC contacts run faster one lane each. Only then are the levels computed: a scalar
  // walk of the contacts in island order (lane b of lastv: 1 + the level of the last contact
  // touching body b).
  const bool big_isl = __builtin_amdgcn_ballot_w64(lsz > kLevelsMinIsland) != 0ull;
  lvl_path = lvl_path && big_isl;
  // More than 64 touching contacts (converged flocks: islands of 60-100 contacts, tests/gs_depth.py):
  // the same levels with S = 2 or 4 contacts per lane (WideLevels below); the per-island lanes
  // would walk such an island serially, ~470 cycles per contact update
  const bool lvl_wide = T > 64 && big_isl;
  const bool skip_isl = lvl_path || lvl_wide;  // no per-island lanes: the level paths solve every island
  // ---- integrate positions --------------------------------------------------
  float cx = p.x, cy = p.y;
  auto integrate_positions = [&]() {
    if (act) {
      vx = s_v[lane].x;
      vy = s_v[lane].y;
      const float tx = P.dt * vx, ty = P.dt * vy;
      if (tx * tx + ty * ty > kMaxTranslation * kMaxTranslation) {
        const float ratio = kMaxTranslation / sqrtf(tx * tx + ty * ty);
        vx = vx * ratio;
        vy = vy * ratio;
      }
      cx = cx + P.dt * vx;
      cy = cy + P.dt * vy;
      s_c[lane] = make_float2(cx, cy);
    }
  };
  if (lvl_wide) {
    // the whole solve per slot count, so that the two variants' registers never meet
    int* s_pmin = reinterpret_cast<int*>(s_imin);  // as in the one-slot level path
    const int Tw = s_ic[nisl];  // contacts in islands (= T unless TDM's degree cap cut edges)
    auto wide = [&](auto sc, auto rc) {
      constexpr int S = decltype(sc)::value;
      constexpr bool REG = decltype(rc)::value;
      WideLevels wl;
      wl.template init<S, REG>(lane, Tw, nisl, s_ord, s_tab, s_tnx, s_tny, s_tln, s_tlt, s_ic, s_tm);
      wl.template velocity<S, REG>(P, s_v, s_tnx, s_tny, s_tln, s_tlt, mA, mB, kmass, friction);
      __syncthreads();
      STAMP(5);
      integrate_positions();
      __syncthreads();
      STAMP(6);
      wl.template position<S>(P, lane, nisl, s_c, s_pmin, s_isolved, mA, mB);
      wave_lds_sync();
      if (lane < nisl) s_imin[lane] = 0xffffffffu;  // island sleep decision below
    };
    if (Tw <= 128) wide(IntC<2>{}, BoolC<true>{});
    else wide(IntC<4>{}, BoolC<false>{});
  } else {
    if (lvl_path) {
      const uint32_t tabv = lane < T ? s_tab[lane] : 0u;
      uint32_t lastv = 0u;
      for (int k = 0; k < T; ++k) {
        const uint32_t ab = (uint32_t)__builtin_amdgcn_readlane(tabv, __builtin_amdgcn_readlane(ordv, k));
        const int a = ab & 0xffffu, bb = ab >> 16;
        const int l = max(__builtin_amdgcn_readlane(lastv, a), __builtin_amdgcn_readlane(lastv, bb));
        lastv = writelane_m0(l + 1, a, lastv);
        lastv = writelane_m0(l + 1, bb, lastv);
        lvlv = writelane_m0(l, k, lvlv);
      }
      int isl = 0;  // island of contact `lane`: the islands whose first contact is at or before it
      for (int I = 1; I < nisl; ++I) isl += (int)s_ic[I] <= lane ? 1 : 0;
      kislv = (uint32_t)isl;
    }
    // level path: lane k holds contact k (island order) for the whole solve
    const bool lhas = lvl_path && lane < T;
    const int lvl = (int)lvlv, lisl = (int)kislv;
    int dmulti = 0;  // levels of the islands with >= 2 contacts (0: only single-contact islands)
    int lt_ = 0, la = 0, lb = 0;
    float lnx = 0.0f, lny = 0.0f, lln = 0.0f, llt = 0.0f;
    if (lvl_path) {
      const int c0 = lhas ? (int)s_ic[lisl] : 0, c1 = lhas ? (int)s_ic[lisl + 1] : 0;
      dmulti = wave_max(lhas && c1 - c0 >= 2 ? lvl + 1 : 0);
      if (lhas) {
        lt_ = (int)ordv;
        const uint32_t ab = s_tab[lt_];
        la = ab & 0xffffu;
        lb = ab >> 16;
        lnx = s_tnx[lt_];
        lny = s_tny[lt_];
        lln = s_tln[lt_];
        llt = s_tlt[lt_];
      }
    }
    // between level steps: the next lanes see this step's LDS writes (wave_lds_sync)
    auto level_sync = [&]() { wave_lds_sync(); };
    if (lvl_path && dmulti == 0) {  // single-contact islands only: every pass in registers
      if (lhas) {
        const float2 vA0 = s_v[la], vB0 = s_v[lb];
        float vAx = vA0.x, vAy = vA0.y, vBx = vB0.x, vBy = vB0.y;
        if (P.warm_starting) warm_start_contact(vAx, vAy, vBx, vBy, lnx, lny, lln, llt, mA, mB);
        for (int it = 0; it < P.vel_iters; ++it)
          solve_velocity_contact(vAx, vAy, vBx, vBy, lnx, lny, lln, llt, mA, mB, kmass, friction);
        s_v[la] = make_float2(vAx, vAy);
        s_v[lb] = make_float2(vBx, vBy);
      }
    } else if (lvl_path) {
      // the warm-start pass and the velocity passes as separate loops: no branch inside a level step.
      // Every lane runs every level step, the lanes outside the level on their own dummy slot in
      // s_tm (the DFS masks: dead until the next step's Collide), so a level step has no exec-mask
      // branch; only the level's lanes keep their impulses
      float2* const pdd = reinterpret_cast<float2*>(s_tm) + lane;
      float2* const pda = lhas ? s_v + la : pdd;
      float2* const pdb = lhas ? s_v + lb : pdd;
      const int mylvl = lhas ? lvl : -1;
      auto lpass = [&](auto warm) {
        // the next level's addresses are selected while this level solves (off the read's path);
        // two level steps per iteration (no register rotation or back-edge per level, as kernel B)
        float2* pa = mylvl == 0 ? pda : pdd;
        float2* pb = mylvl == 0 ? pdb : pdd;
        auto step = [&](bool onc, bool onn) {
          float nl = lln, nt = llt;
          const float2 vA0 = *pa, vB0 = *pb;
          float2* const na = onn ? pda : pdd;
          float2* const nb = onn ? pdb : pdd;
          float vAx = vA0.x, vAy = vA0.y, vBx = vB0.x, vBy = vB0.y;
          if constexpr (decltype(warm)::value) warm_start_contact(vAx, vAy, vBx, vBy, lnx, lny, nl, nt, mA, mB);
          else solve_velocity_contact(vAx, vAy, vBx, vBy, lnx, lny, nl, nt, mA, mB, kmass, friction);
          *pa = make_float2(vAx, vAy);
          *pb = make_float2(vBx, vBy);
          lln = onc ? nl : lln;
          llt = onc ? nt : llt;
          pa = na;
          pb = nb;
          level_sync();
        };
        int l = 0;
        for (; l + 1 < dmulti; l += 2) {
          step(mylvl == l, mylvl == l + 1);
          step(mylvl == l + 1, mylvl == l + 2);
        }
        for (; l < dmulti; ++l) step(mylvl == l, mylvl == l + 1);
      };
      if (P.warm_starting) lpass(BoolC<true>{});
      for (int it = 0; it < P.vel_iters; ++it) lpass(BoolC<false>{});
    }
    if (lhas) {
      s_tln[lt_] = lln;
      s_tlt[lt_] = llt;
    }
    for (int I = skip_isl ? W : lane; I < nisl; I += W) {
      const int c0 = s_ic[I], c1 = s_ic[I + 1];
      if (c1 - c0 == 1 && !krec_wave) {
        const int t = s_ord[c0];
        const uint32_t ab = s_tab[t];
        const int a = ab & 0xffffu, b = ab >> 16;
        const float nx = s_tnx[t], ny = s_tny[t];
        float ln = s_tln[t], ltg = s_tlt[t];
        const float2 vA0 = s_v[a], vB0 = s_v[b];
          float vAx = vA0.x, vAy = vA0.y, vBx = vB0.x, vBy = vB0.y;
        if (P.warm_starting) warm_start_contact(vAx, vAy, vBx, vBy, nx, ny, ln, ltg, mA, mB);
        for (int it = 0; it < P.vel_iters; ++it)
          solve_velocity_contact(vAx, vAy, vBx, vBy, nx, ny, ln, ltg, mA, mB, kmass, friction);
        s_v[a] = make_float2(vAx, vAy);
        s_v[b] = make_float2(vBx, vBy);
        s_tln[t] = ln;
        s_tlt[t] = ltg;
        continue;
      }
      if (c1 - c0 <= KREC) {  // records and impulses in registers, body velocities in LDS (see KREC)
        const int L = c1 - c0;
        int rt[KRECA];
        uint32_t rab_[KRECA];
        float rnx[KRECA], rny[KRECA], rln[KRECA], rlt[KRECA];
  #pragma unroll
        for (int q = 0; q < KREC; ++q) rt[q] = q < L ? s_ord[c0 + q] : 0;
  #pragma unroll
        for (int q = 0; q < KREC; ++q) {
          rab_[q] = s_tab[rt[q]];
          rnx[q] = s_tnx[rt[q]];
          rny[q] = s_tny[rt[q]];
          rln[q] = s_tln[rt[q]];
          rlt[q] = s_tlt[rt[q]];
        }
        if (P.warm_starting) {
  #pragma unroll
          for (int q = 0; q < KREC; ++q) {
            if (q < L) {
              const int a = rab_[q] & 0xffffu, b = rab_[q] >> 16;
              const float2 vA0 = s_v[a], vB0 = s_v[b];
          float vAx = vA0.x, vAy = vA0.y, vBx = vB0.x, vBy = vB0.y;
              warm_start_contact(vAx, vAy, vBx, vBy, rnx[q], rny[q], rln[q], rlt[q], mA, mB);
              s_v[a] = make_float2(vAx, vAy);
              s_v[b] = make_float2(vBx, vBy);
            }
          }
        }
        for (int it = 0; it < P.vel_iters; ++it) {
  #pragma unroll
          for (int q = 0; q < KREC; ++q) {
            if (q < L) {
              const int a = rab_[q] & 0xffffu, b = rab_[q] >> 16;
              const float2 vA0 = s_v[a], vB0 = s_v[b];
          float vAx = vA0.x, vAy = vA0.y, vBx = vB0.x, vBy = vB0.y;
              solve_velocity_contact(vAx, vAy, vBx, vBy, rnx[q], rny[q], rln[q], rlt[q], mA, mB, kmass, friction);
              s_v[a] = make_float2(vAx, vAy);
              s_v[b] = make_float2(vBx, vBy);
            }
          }
        }
  #pragma unroll
        for (int q = 0; q < KREC; ++q) {
          if (q < L) {
            s_tln[rt[q]] = rln[q];
            s_tlt[rt[q]] = rlt[q];
          }
        }
        continue;
      }
      if (P.warm_starting) {
        for (int k = c0; k < c1; ++k) {
          const int t = s_ord[k];
          const uint32_t ab = s_tab[t];
          const int a = ab & 0xffffu, b = ab >> 16;
          const float2 vA0 = s_v[a], vB0 = s_v[b];
          float vAx = vA0.x, vAy = vA0.y, vBx = vB0.x, vBy = vB0.y;
          warm_start_contact(vAx, vAy, vBx, vBy, s_tnx[t], s_tny[t], s_tln[t], s_tlt[t], mA, mB);
          s_v[a] = make_float2(vAx, vAy);
          s_v[b] = make_float2(vBx, vBy);
        }
      }
      for (int it = 0; it < P.vel_iters; ++it) {
        for (int k = c0; k < c1; ++k) {
          const int t = s_ord[k];
          const uint32_t ab = s_tab[t];
          const int a = ab & 0xffffu, b = ab >> 16;
          const float2 vA0 = s_v[a], vB0 = s_v[b];
          float vAx = vA0.x, vAy = vA0.y, vBx = vB0.x, vBy = vB0.y;
          float ln = s_tln[t], ltg = s_tlt[t];
          solve_velocity_contact(vAx, vAy, vBx, vBy, s_tnx[t], s_tny[t], ln, ltg, mA, mB, kmass, friction);
          s_v[a] = make_float2(vAx, vAy);
          s_v[b] = make_float2(vBx, vBy);
          s_tln[t] = ln;
          s_tlt[t] = ltg;
        }
      }
    }
    __syncthreads();
    STAMP(5);
    integrate_positions();
    __syncthreads();
    STAMP(6);

    // ---- position iterations, one lane per island ------------------------------
    if (lvl_path) {
      // per island: the pass's minimum separation (order-preserving int keys); s_imin holds them
      // until the island sleep decision below re-initialises it (one LDS array fewer keeps 17
      // waves' LDS per CU: 4096 envs stay a single dispatch round with slack)
      int* s_pmin = reinterpret_cast<int*>(s_imin);
      if (dmulti == 0) {  // single-contact islands: lane k runs island k's passes in registers
        if (lhas) {
          int solved = 0;
          const float2 cA0 = s_c[la], cB0 = s_c[lb];
          float cAx = cA0.x, cAy = cA0.y, cBx = cB0.x, cBy = cB0.y;
          for (int it = 0; it < P.pos_iters; ++it) {
            const float sep = solve_position_contact(cAx, cAy, cBx, cBy, P.radius, mA, mB);
            if (bmin(0.0f, sep) >= -3.0f * kLinearSlop) {
              solved = 1;
              break;
            }
          }
          s_c[la] = make_float2(cAx, cAy);
          s_c[lb] = make_float2(cBx, cBy);
          s_isolved[lisl] = (uint8_t)solved;
        }
      } else {
        // passes over the levels; an island leaves after the first pass whose minimum separation
        // (from 0) is >= -3 linearSlop (b2Island::Solve)
        const unsigned long long islm = nisl >= 64 ? ~0ull : ((1ull << nisl) - 1ull);
        unsigned long long done = 0ull;
        for (int it = 0; it < P.pos_iters && done != islm; ++it) {
          if (lane < nisl) s_pmin[lane] = __float_as_int(0.0f);
          level_sync();
          // branch-free level steps as in the velocity passes: the lanes outside the level (or of
          // an island that has left) correct their own dummy slot in s_tm and take their minimum
          // into its first word
          const int mylvl = (lhas && !((done >> lisl) & 1ull)) ? lvl : -1;
          float2* const pdd = reinterpret_cast<float2*>(s_tm) + lane;
          float2* const pda = lhas ? s_c + la : pdd;
          float2* const pdb = lhas ? s_c + lb : pdd;
          int* const pmd = reinterpret_cast<int*>(pdd);  // a dummy lane's minimum: its own word
          int* const pmi = lhas ? s_pmin + lisl : pmd;
          float2* pa = mylvl == 0 ? pda : pdd;
          float2* pb = mylvl == 0 ? pdb : pdd;
          int* pm = mylvl == 0 ? pmi : pmd;
          auto pstep = [&](bool onn) {
            float2* const na = onn ? pda : pdd;
            float2* const nb = onn ? pdb : pdd;
            int* const nm = onn ? pmi : pmd;
            const float2 cA0 = *pa, cB0 = *pb;
            float cAx = cA0.x, cAy = cA0.y, cBx = cB0.x, cBy = cB0.y;
            const float sep = solve_position_contact(cAx, cAy, cBx, cBy, P.radius, mA, mB);
            *pa = make_float2(cAx, cAy);
            *pb = make_float2(cBx, cBy);
            // order-preserving int of the float for atomicMin
            const int key = __float_as_int(sep) >= 0 ? __float_as_int(sep) : (__float_as_int(sep) ^ 0x7fffffff);
            atomicMin(pm, key);
            pa = na;
            pb = nb;
            pm = nm;
            level_sync();
          };
          int l = 0;
          for (; l + 1 < dmulti; l += 2) {
            pstep(mylvl == l + 1);
            pstep(mylvl == l + 2);
          }
          for (; l < dmulti; ++l) pstep(mylvl == l + 1);
          int km = lane < nisl ? s_pmin[lane] : 0;
          km = km >= 0 ? km : (km ^ 0x7fffffff);
          done |= __builtin_amdgcn_ballot_w64(lane < nisl && !((done >> lane) & 1ull) &&
                                              __int_as_float(km) >= -3.0f * kLinearSlop);
        }
        if (lane < nisl) s_isolved[lane] = (uint8_t)((done >> lane) & 1ull);
      }
      level_sync();
      if (lane < nisl) s_imin[lane] = 0xffffffffu;  // island sleep decision below
    }
    for (int I = skip_isl ? W : lane; I < nisl; I += W) {
      s_imin[I] = 0xffffffffu;  // island sleep decision below
      const int c0 = s_ic[I], c1 = s_ic[I + 1];
      int solved = 0;
      if (c1 - c0 == 1 && !krec_wave) {  // single contact: registers
        const uint32_t ab = s_tab[s_ord[c0]];
        const int a = ab & 0xffffu, b = ab >> 16;
        const float2 cA0 = s_c[a], cB0 = s_c[b];
          float cAx = cA0.x, cAy = cA0.y, cBx = cB0.x, cBy = cB0.y;
        for (int it = 0; it < P.pos_iters; ++it) {
          const float sep = solve_position_contact(cAx, cAy, cBx, cBy, P.radius, mA, mB);
          const float min_sep = bmin(0.0f, sep);
          if (min_sep >= -3.0f * kLinearSlop) {
            solved = 1;
            break;
          }
        }
        s_c[a] = make_float2(cAx, cAy);
        s_c[b] = make_float2(cBx, cBy);
        s_isolved[I] = (uint8_t)solved;
        continue;
      }
      if (c1 - c0 <= KREC) {  // pairs in registers, body positions in LDS (see KREC)
        const int L = c1 - c0;
        uint32_t rab_[KRECA];
  #pragma unroll
        for (int q = 0; q < KREC; ++q) rab_[q] = s_tab[q < L ? s_ord[c0 + q] : 0];
        for (int it = 0; it < P.pos_iters; ++it) {
          float min_sep = 0.0f;
  #pragma unroll
          for (int q = 0; q < KREC; ++q) {
            if (q < L) {
              const int a = rab_[q] & 0xffffu, b = rab_[q] >> 16;
              const float2 cA0 = s_c[a], cB0 = s_c[b];
          float cAx = cA0.x, cAy = cA0.y, cBx = cB0.x, cBy = cB0.y;
              const float sep = solve_position_contact(cAx, cAy, cBx, cBy, P.radius, mA, mB);
              min_sep = bmin(min_sep, sep);
              s_c[a] = make_float2(cAx, cAy);
              s_c[b] = make_float2(cBx, cBy);
            }
          }
          if (min_sep >= -3.0f * kLinearSlop) {
            solved = 1;
            break;
          }
        }
        s_isolved[I] = (uint8_t)solved;
        continue;
      }
      for (int it = 0; it < P.pos_iters; ++it) {
        float min_sep = 0.0f;
        for (int k = c0; k < c1; ++k) {
          const uint32_t ab = s_tab[s_ord[k]];
          const int a = ab & 0xffffu, b = ab >> 16;
          const float2 cA0 = s_c[a], cB0 = s_c[b];
          float cAx = cA0.x, cAy = cA0.y, cBx = cB0.x, cBy = cB0.y;
          const float sep = solve_position_contact(cAx, cAy, cBx, cBy, P.radius, mA, mB);
          min_sep = bmin(min_sep, sep);
          s_c[a] = make_float2(cAx, cAy);
          s_c[b] = make_float2(cBx, cBy);
        }
        if (min_sep >= -3.0f * kLinearSlop) {
          solved = 1;
          break;
        }
      }
      s_isolved[I] = (uint8_t)solved;
    }

  }

  // After the chain a wave with touching contacts stays above the contact-free ones, and one
  // with >= 3 touching contacts (the envs that end last) above those: -2% per step against a
  // single level (profiles/r01/ab2 s24/s25; thresholds 2 and 4, or a third level, did no better).
  if (hasdeg) {
    if (T >= kPrio2T) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(1);
  }
  // ---- per-body sleep clock ---------------------------------------------------
  float ns = 0.0f;
  if (act) {
    const bool moving = vx * vx + vy * vy > kLinearSleepTol * kLinearSleepTol;
    ns = moving ? 0.0f : slp + P.dt;
  }
  __syncthreads();
  STAMP(7);

  // ---- island sleep decision ---------------------------------------------------
  // min sleep time over each island's bodies (b2Island::Solve) by LDS atomicMin on the
  // float bits (sleep times are >= 0, so their bit patterns order as the values)
  const bool inisl = act && deg > 0;
  const int myisl = inisl ? s_bisl[lane] : 0;
  if (inisl) atomicMin(&s_imin[myisl], __float_as_uint(ns));
  __syncthreads();
  bool sleepnow = false;
  if (act) {
    sleepnow = inisl ? (__uint_as_float(s_imin[myisl]) >= kTimeToSleep && s_isolved[myisl])
                     : (ns >= kTimeToSleep && P.pos_iters > 0);
  }
  STAMP(8);

  // ---- SynchronizeFixtures: fat-AABB update ------------------------------------
  float4 fn = fo;
  if (act) {
    cx = s_c[lane].x;
    cy = s_c[lane].y;
    const float r = P.radius;
    const float c0x = p.x, c0y = p.y;
    const float lox = bmin(c0x - r, cx - r), loy = bmin(c0y - r, cy - r);
    const float hix = bmax(c0x + r, cx + r), hiy = bmax(c0y + r, cy + r);
    const bool contains = fo.x <= lox && fo.y <= loy && hix <= fo.z && hiy <= fo.w;
    if (!contains) {
      fn = make_float4(lox - kAabbExtension, loy - kAabbExtension, hix + kAabbExtension, hiy + kAabbExtension);
      const float dx = kAabbMultiplier * (cx - c0x), dy = kAabbMultiplier * (cy - c0y);
      if (dx < 0.0f) fn.x += dx; else fn.z += dx;
      if (dy < 0.0f) fn.y += dy; else fn.w += dy;
    }
    if (sleepnow) {
      vx = 0.0f;
      vy = 0.0f;
      ns = 0.0f;
    }
  }
  {
    // per-agent record for the all-pairs sweep; lanes >= N hold a dummy whose AABB
    // overlaps nothing and whose position is infinitely far away
    PairRec r;
    r.fn = act ? fn : make_float4(__builtin_inff(), __builtin_inff(), -__builtin_inff(), -__builtin_inff());
    r.c = act ? make_float2(cx, cy) : make_float2(__builtin_inff(), __builtin_inff());
    r.pad = make_float2(0.0f, 0.0f);
    s_pj[lane] = r;
  }
  __syncthreads();  // s_pj and final s_c visible to every lane
  STAMP(9);

  // ---- contact set, new pairs, nearest neighbour ---------------------------------
  // The old list IS Ov(F_{t-1}), so only the new fat AABBs are tested here:
  //   world.contacts after the step = Ov(F_{t-1}) U Ov(F_t)        
  //   FindNewContacts creates        Ov(F_t) \ Ov(F_{t-1})
  // Agent j's record arrives by LDS broadcast; each lane accumulates its own partner
  // row one bit per record (2 VALU: compare into VCC, add-with-carry). The sweep is
  // fully unrolled over NCAP >= N records (lanes >= N hold dummies that overlap
  // nothing and are infinitely far), so j is a compile-time constant, and the AABB /
  // distance differences run as packed float2 ops (each lane-wise result is the same
  // IEEE op as scalar). The ballot + v_writelane form of the row costs 0.5% more.
  const unsigned long long valid = livem;
  SweepState sw;
  sw.ov_lo = 0u;
  sw.ov_hi = 0u;
  sw.best = __builtin_inff();
  sw.bj = lane == 0 ? 1 : 0;
  if constexpr (NCAP == 64 && !kT) {  // two interleaved chains
    constexpr int AH2 = 2 * kSweepAhead;  // records in flight (two per step)
    SweepState2 s2;
    s2.ov_lo = 0u;
    s2.ov_hi = 0u;
    s2.best_a = __builtin_inff();
    s2.best_b = __builtin_inff();
    s2.bj_a = lane == 0 ? 1 : 0;
    s2.bj_b = 32;
    SweepRec win[AH2];
#pragma unroll
    for (int k = 0; k < AH2; ++k) win[k] = load_rec(s_pj, (k & 1) ? 32 + (k >> 1) : (k >> 1));
    sweep2_step<0, AH2, SCAL>(s_pj, win, mk2(fn.x, fn.y), mk2(fn.z, fn.w), mk2(cx, cy), s2);
    sw.ov_lo = s2.ov_lo;
    sw.ov_hi = s2.ov_hi;
    const bool upper = s2.best_b < s2.best_a;  // the lower half wins ties (lower indices)
    sw.best = upper ? s2.best_b : s2.best_a;
    sw.bj = upper ? s2.bj_b : s2.bj_a;
  } else {
    SweepRec win[kSweepAhead];
#pragma unroll
    for (int k = 0; k < kSweepAhead; ++k) win[k] = load_rec(s_pj, k);
    sweep_step<0, NCAP, !kT>(s_pj, win, mk2(fn.x, fn.y), mk2(fn.z, fn.w), mk2(cx, cy), valid, lane, sw);
  }
  const float best = sw.best;
  const int bj = sw.bj;
  const uint32_t ov_lo = __builtin_bitreverse32(sw.ov_lo), ov_hi = __builtin_bitreverse32(sw.ov_hi);
  unsigned long long myov = (((unsigned long long)ov_hi << 32) | ov_lo) & valid;
  myov &= ~(1ull << lane);
  const unsigned long long oldm = (unsigned long long)s_oldm[2 * lane] | ((unsigned long long)s_oldm[2 * lane + 1] << 32);
  const bool coll = act && ((myov | oldm) != 0ull);
  const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  const unsigned long long newmask = act ? (myov & ~oldm & above) : 0ull;
  STAMP(10);

  // ---- next ordered list: new pairs (desc) ++ surviving old pairs --------------
  uint32_t* ocab = B.cab[nxt] + (size_t)e * C;
  float2* ocimp = B.cimp[nxt] + (size_t)e * C;
  const int nnew = write_new_pairs(lane, newmask, ocab, ocimp, C);
  int kept = 0, Tr = 0;
  for (int c = 0; c * W < M; ++c) {
    const int k = c * W + lane;
    uint32_t ab = 0u;
    if (c < RCH) {
#pragma unroll
      for (int q = 0; q < RCH; ++q)
        if (q == c) ab = rab[q];
    } else if (k < M) {
      ab = cab[k];
    }
    bool keep = false;
    const bool touch = (tbits >> c) & 1u;
    if (k < M) {
      const int a = ab & 0xffffu, b = ab >> 16;
      keep = overlap(s_pj[a].fn, s_pj[b].fn);
    }
    const unsigned long long mt = __ballot(touch), mk = __ballot(keep);
    const int trank = Tr + __popcll(mt & lt);
    const int krank = kept + __popcll(mk & lt);
    Tr += __popcll(mt);
    kept += __popcll(mk);
    if (keep) {
      const int w = nnew + krank;
      if (w < C) {
        float2 l = make_float2(0.0f, 0.0f);
        if (touch && trank < TCAP) l = make_float2(s_tln[trank], s_tlt[trank]);
        st_g<kState>(ocab + w, ab);
        st_g<kState>(ocimp + w, l);
      }
    }
  }
  int total = nnew + kept;
  if (total > C) {
    status |= MACM_ST_CONTACT_OVERFLOW;
    total = C;
  }
  STAMP(11);

  // ---- rewards (mvmnt.py:160-179) and obs (mvmnt.py:181-222) -------------------
  float rew = 0.0f;
  if constexpr (!kT) {
    if (act) {
      const float tdx = tg.x - cx, tdy = tg.y - cy;  // target - agent.body.position
      const float td2 = tdx * tdx + tdy * tdy;       // b2DistanceSquared(target, position)
      const double d = sqrt((double)td2);
      if (coll) rew = -1.0f;
      else if (P.reward_mode == MACM_REWARD_LINEAR) rew = (float)((-d / 35) + 1);
      else rew = (d < P.reward_radius) ? 1.0f : 0.0f;
      st_g<kOut>(rew_out + ag, rew);
      if (coll_out) st_g<kOut>(coll_out + ag, (uint8_t)(coll ? 1 : 0));
      if (nbr_out) st_g<kOut>(nbr_out + ag, (int32_t)bj);
      if (obs) {
        const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
        const float2 cn = s_c[bj];
        const float rx = cn.x - cx, ry = cn.y - cy;
        write_obs<OT>(obs + ag * od, P.coord, ang, best, rx, ry, tdx, tdy, td2);
      }
      // ---- state write-back ----
      st_g<kState>(B.pos + ag, make_float2(cx, cy));
      st_g<kState>(B.vel + ag, make_float2(vx, vy));
      st_g<kState>(B.angle + ag, ang);
      st_g<kState>(B.fat + ag, fn);
      st_g<kState>(B.sleep + ag, ns);
    }
  } else {
    // ---- TDM state write-back + TDM.get_obs (combat.py:166-167, 206-227) -------
    if (lane < N) {
      if (act) {  // in the physics step
        B.pos[ag] = make_float2(cx, cy);
        B.vel[ag] = make_float2(vx, vy);
        B.fat[ag] = fn;
        B.sleep[ag] = ns;
      }
      if (act0) {  // acted this step (possibly died after acting)
        B.angle[ag] = ang;
        TB.cd_atk[ag] = cda;
        TB.cd_mov[ag] = cdm;
      }
      TB.health[ag] = hp;  // the stale listener can damage dead bodies too
      TB.alive[ag] = act ? 1 : 0;
      if (TB.health_out) TB.health_out[ag] = hp;
      if (TB.alive_out) TB.alive_out[ag] = act ? 1 : 0;
    }
    s_ang[lane] = ang;
    __syncthreads();
    if (TB.snap_out) {  // the split observation: the pose snapshot tdm_observe_snap observes
      if (lane < N) {
        const float2 c = s_c[lane];
        st_wt4(TB.snap_out + ag, make_float4(c.x, c.y, ang, act ? 1.0f : 0.0f));  // write-through: the tail observation
      }
    } else {
      const size_t rows = (size_t)e * N * (N - 1);
      OT* const obs_e = obs ? obs + rows * 4 : nullptr;
      uint8_t* const mask_e = TB.mask_out ? TB.mask_out + rows : nullptr;
      bool staged = false;
      if constexpr (sizeof(OT) == 4) {
        if (tdm_obs_rb_stage_bytes(N) <= (int)sizeof(Pool)) {  // the contact arrays are dead here
          tdm_obs_rowblocks<OT>(obs_e, mask_e, N, lane, livem, TP, s_c, s_ang, reinterpret_cast<float4*>(&s_pool));
          staged = true;
        }
      }
      if (!staged) tdm_obs_pairs<OT>(obs_e, mask_e, N, lane, livem, TP, s_c, s_ang);
    }
  }
  STAMP(12);

  // ---- per-env bookkeeping + counters (no cross-env atomics) -------------------
  const unsigned long long mst1 = __ballot(status & 1), mst2 = __ballot(status & 2), mst4 = __ballot(status & 4);
  unsigned long long c1 = 0ull, c2 = 0ull;
  int alive_teams = 0, last_team = -1;
  double rsum = 0.0;
  if constexpr (!kT) {
    c1 = __popcll(__ballot(act && coll));        // collided agent-steps
    c2 = __popcll(__ballot(act && rew > 0.0f));  // positive-reward agent-steps
    // linear rewards only: a binary step sums to c2 - c1 exactly (macm_world_reward_sums)
    if (P.reward_mode == MACM_REWARD_LINEAR) rsum = wave_pairwise_sum((double)rew);  // lanes >= N: rew = +0.0
  } else {
    c1 = __popcll(att_m);               // melee attacks
    c2 = __popcll(alive0_m & ~livem);   // deaths
    const int myteam = tdm_team_of(TP, lane);
    for (int t = 0; t < TP.n_teams; ++t)
      if (__ballot(act && myteam == t)) {
        ++alive_teams;
        last_team = t;
      }
  }
  if (lane == 0) {
    const double tp = time_passed + P.inv_hz;  // time_passed += 1/hz
    uint8_t dn = tp > P.time_limit ? 1 : 0;
    if constexpr (kT) {
      // combat.py:172-182: done latches; winner = the last team standing
      int win = win_prev;
      if (done_prev) dn = 1;
      if (alive_teams == 1) {
        dn = 1;
        win = last_team;
      }
      if (alive_teams == 0) dn = 1;
      TB.winner[e] = win;
      if (TB.winner_out) TB.winner_out[e] = win;
      TB.listener[e] = lis;
    }
    B.time_passed[e] = tp;
    B.done[e] = dn;
    if (done_out) done_out[e] = dn;
    B.step_count[e] = step_count + 1;
    B.ccount[nxt][e] = total;
    const int st = (mst1 ? 1 : 0) | (mst2 ? 2 : 0) | (mst4 ? 4 : 0);
    if (st) {
      B.status[e] = st_prev | st;
      report_status(B, st);
    }
    const unsigned long long c0 = kT ? (unsigned long long)__popcll(alive0_m) : (unsigned long long)N;
    ulonglong2* ec = reinterpret_cast<ulonglong2*>(B.env_counters + (size_t)e * 4);
    ec[0] = make_ulonglong2(ctr[0] + c0, ctr[1] + c1);
    ec[1] = make_ulonglong2(ctr[2] + c2, ctr[3] + (unsigned long long)dn);
    if constexpr (!kT) {
      if (P.reward_mode == MACM_REWARD_LINEAR) add_reward_sum(B, e, rsum);
    }
  }
  STAMP(13);
#ifdef MACM_TIMELINE
  {
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime(), c1t = __builtin_amdgcn_s_memtime();
    const unsigned long long hw = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned long long xcc = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    if (lane == 0) {
      unsigned long long* st = B.stamps + (size_t)e * 16;
      st[0] = tl_rt0;
      st[1] = tl_c0;
      st[2] = hw | (xcc << 32);
      st[3] = rt1;
      st[4] = c1t;
    }
  }
#endif
  STAMP_STAT(14, (unsigned long long)T | ((unsigned long long)nisl << 16) | ((unsigned long long)M << 32));
#ifdef MACM_STAMPS
  STAMP_STAT(15, (unsigned long long)s_stat_maxisl | ((unsigned long long)total << 32));
#endif
}

#ifdef MACM_ROLLOUT_TU

// nsteps consecutive steps of env blockIdx.x in one launch (macm_world_rollout): actions of step k
// at actions + k * astride bytes ([K, E, N, A]), outputs overwritten each step (the last step's
// remain) or, with traj, step k's outputs at row k of [K, ...] buffers (macm_world_rollout_traj),
// counters accumulated. Each env's wave runs its own steps back to back, so no env waits at a
// launch boundary for the slowest env of the batch. Every step reads only what this wave
// wrote in the step before: a workgroup-scope fence completes its stores before the next step's
// loads; the barrier orders the LDS reuse. This part is compiled in its own translation unit
// (flock_rollout_w64.hip, -mllvm -disable-machine-licm): with the step inside a loop, machine
// LICM hoists the f64 polynomial constants of the trig and atan2 code out of it and the
// register allocator spills them (327 VGPRs of spills; none without the hoisting).
// The lane index is made opaque to the compiler in TDM rollouts only (Flock rollouts: measured no
// better, round 4).
template <typename OT>
struct RolloutArgs {  // the kernel's only argument (kernarg offset 0)
  StepParams P;
  WorldBuffers B;
  TdmParams TP;
  TdmBuffers TB;
  const void* actions;
  OT* obs;
  int32_t* nbr_out;
  float* rew_out;
  uint8_t* coll_out;
  uint8_t* done_out;
  unsigned long long astride;
  int cur;
  int nsteps;
  // closed loop (macm_world_rollout_bots): every step reads its actions here and the device bot
  // (bots.hpp) writes the next step's from the observation this step wrote; NULL: actions[k]
  uint8_t* policy_act;
  // trajectory form: every output (and, in the closed loop, the bot's actions: [K + 1, E, N, A],
  // step k reading row k and writing row k + 1) advances one row per step
  int traj;
  // A balanced launch steps envs order[sched_off + blockIdx.x]; sched_off is 0 since the solo split
  // was removed (round 6), and kept with `reserved` so the kernel's argument layout (and with it its
  // register allocation) stays the measured one: without them the driver window ran 1.1% slower, with
  // them 0.3% (in noise) against the library before the removal (profiles/r06/abtests/cleanup/).
  int sched_off;
  // the tail observation (TailObs; TDM trajectory rollouts, macm_capi tdm_tail_obs): its counters and
  // ready words, and this launch's tag (0: off; blocks beyond n_envs then do not exist)
  unsigned long long* tail_ctl;
  unsigned int tail_tag;
  int tail_k0;  // the first step observed in the tail (0: all); the steps before observe in the step
};

// [K, ...] row k of an output (trajectory form); NULL stays NULL
template <typename T>
__device__ __forceinline__ T* traj_row(T* p, size_t k, size_t per_step) {
  return p ? p + k * per_step : p;
}

// Load balancing of a rollout launch (round 4). A rollout keeps each env on one wave for all K
// steps, so the launch ends with the wave of the heaviest env (a dense or converged flock whose
// Gauss-Seidel chain is several times the mean), and two or three such envs that land on one SIMD
// slow each other's latency-bound chains. Before the rollout, rollout_sched orders the envs by
// their contact-list size (the work of the step's chain grows with it), heaviest first, and wave b
// of the rollout steps env order[b]: the dispatcher places one wave per SIMD before the second, so
// the heaviest envs start one per SIMD. An env's results do not depend on its wave. Measured
// (profiles/r04/abtests/roll_balance): M closed loop 160 -> 148 us per step; the scheduling kernel
// costs ~6 us per launch (+0.3 us per step of a 20-step rollout, no gain there), so rollouts shorter
// than kRollBalanceMinSteps keep wave b on env b. Claiming envs by SIMD id at the wave's start
// (3 device-scope atomics per wave on two counters) balanced as well but cost ~50 us per launch.
constexpr int kRollBalanceMinSteps = 32;
constexpr int kSchedMaxSize = 4095;

// order[0..E): the envs by descending contact-list size (ccount, clamped to C); one workgroup.
// reset2: the workgroup step's handoff counters (Handoff::ctr), zeroed for the step (or NULL)
__global__ __launch_bounds__(1024) void rollout_sched(const uint32_t* __restrict__ ccount, uint32_t* __restrict__ order,
                                                     int E, int C, unsigned int* reset2 = nullptr) {
  extern __shared__ uint32_t s_h[];  // [C + 1] envs per list size, then the order's starts
  __shared__ int s_scan[32];
  const int tid = threadIdx.x, BS = blockDim.x;
  if (reset2 && tid < 2) reset2[tid] = 0u;
  for (int i = tid; i <= C; i += BS) s_h[i] = 0u;
  __syncthreads();
  for (int e = tid; e < E; e += BS) atomicAdd(&s_h[max(0, min((int)ccount[e], C))], 1u);
  __syncthreads();
  {  // starts in descending size: thread t owns sizes C - t per .. C - t per - per + 1
    const int per = (C + 1 + BS - 1) / BS, hi = C - tid * per, lo = max(-1, hi - per);
    int sum = 0;
    for (int c = hi; c > lo; --c) sum += (int)s_h[c];
    int run;
    spill::block_scan_excl(sum, run, s_scan);
    for (int c = hi; c > lo; --c) {
      const int n = (int)s_h[c];
      s_h[c] = (uint32_t)run;
      run += n;
    }
  }
  __syncthreads();
  for (int e = tid; e < E; e += BS) order[atomicAdd(&s_h[max(0, min((int)ccount[e], C))], 1u)] = (uint32_t)e;
}

// A balanced rollout's heaviest envs in waves that own their SIMD, on a stream of their own ("solo"
// waves, round 5), measured slower and were removed in round 6 (profiles/r05/abtests/).
template <int MODE, int NCAP, typename OT, bool SCAL = false>
__global__ __launch_bounds__(W) __attribute__((amdgpu_waves_per_eu(4))) void env_rollout_w64(RolloutArgs<OT> A0) {
  const int nsteps = A0.nsteps;
  const bool bal = A0.B.sched && nsteps >= kRollBalanceMinSteps;  // as in launch_roll
  // TDM tail observation: blocks beyond the envs only observe (TailObs)
  const bool phys = MODE != kTdm || (int)blockIdx.x < A0.P.n_envs;
  const int env = bal && phys ? (int)A0.B.sched[A0.sched_off + blockIdx.x] : (int)blockIdx.x;
  // (the body gets &tl itself in TDM, never a select of it, so that tl stays in registers; ctl NULL = off)
  const int nq = gridDim.x < (unsigned)kTailQ ? (int)gridDim.x : kTailQ;
  TailObs tl{};  // every field named: an initializer list in declaration order hid a misplaced field once
  tl.ctl = A0.tail_tag ? A0.tail_ctl : nullptr;
  tl.tag = A0.tail_tag;
  tl.nsteps = nsteps - A0.tail_k0;
  tl.k = 0;
  tl.worker = false;
  tl.more = true;
  tl.q = (int)(blockIdx.x % nq);
  tl.left = 1;
  tl.r = 0;
  tl.r_end = 0;
  tl.nq = nq;
  const int ksteps = phys ? nsteps : 0;
  for (int k = 0; k < ksteps; ++k) {
    // each step reads its parameters from the kernel arguments afresh, through a pointer the
    // compiler cannot see through, so nothing derived from them stays live across the loop
    const __attribute__((address_space(4))) RolloutArgs<OT>* ka =
        (const __attribute__((address_space(4))) RolloutArgs<OT>*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const RolloutArgs<OT>& A = *(const RolloutArgs<OT>*)ka;
    const int N = A.P.n_agents, lane = threadIdx.x;
    const size_t EN = (size_t)A.P.n_envs * N;
    const size_t kr = A.traj ? (size_t)k : 0;  // output row of this step
    const size_t od = MODE == kTdm ? (size_t)(N - 1) * 4 : (A.P.coord == MACM_COORD_CARTESIAN ? 6 : 4);
    OT* const obs = traj_row(A.obs, kr, EN * od);
    TdmBuffers TB = A.TB;
    if constexpr (MODE == kTdm) {
      TB.mask_out = traj_row(TB.mask_out, kr, EN * (N - 1));
      TB.health_out = traj_row(TB.health_out, kr, EN);
      TB.alive_out = traj_row(TB.alive_out, kr, EN);
      TB.winner_out = traj_row(TB.winner_out, kr, (size_t)A.P.n_envs);
      // the tail observation: snapshots of the last nsteps - tail_k0 steps only ([K - k0, E, N]); the
      // steps before observe in the step (snap_out NULL)
      TB.snap_out = A.tail_tag ? (k >= A.tail_k0 ? traj_row(TB.snap_out, (size_t)(k - A.tail_k0), EN) : nullptr)
                               : traj_row(TB.snap_out, kr, EN);
    }
    const size_t abytes = MODE == kTdm ? 4 : 3;  // closed loop: uint8 actions per agent
    uint8_t* const pol_in = A.policy_act ? A.policy_act + kr * EN * abytes : nullptr;
    __builtin_amdgcn_s_setprio(0);  // as at a launch: the chain raises it again
    // The lane index, opaque to the compiler inside the loop: else every lane-derived address and
    // mask of the step is hoisted out of it and held across all K steps. The TDM step then ran out
    // of its 128 VGPRs and kept 7 of them in scratch, re-read every step (rollout: 28 B per lane).
    int sl = (int)threadIdx.x;
    if constexpr (MODE == kTdm) asm volatile("" : "+v"(sl));
    tl.k = k - A0.tail_k0;
    step_w64_body<MODE, NCAP, OT, SCAL>(A.P, A.B, A.TP, TB, A.cur ^ (k & 1),
                                        pol_in ? pol_in : static_cast<const unsigned char*>(A.actions) + (size_t)k * A.astride,
                                        obs, traj_row(A.nbr_out, kr, EN), traj_row(A.rew_out, kr, EN),
                                        traj_row(A.coll_out, kr, EN), traj_row(A.done_out, kr, (size_t)A.P.n_envs),
                                        env, sl, MODE == kTdm ? &tl : nullptr);
    // the next step reads only what this wave wrote: workgroup scope (this CU's L1 and its XCD's L2)
    // suffices; agent scope would write back and invalidate the L2 every step (5x slower, measured)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __syncthreads();
    if (pol_in) {  // every agent row, as the bots kernel over all E x N rows
      uint8_t* const pol_out = A.traj ? pol_in + EN * abytes : pol_in;
      if (lane < N) {
        const size_t row = (size_t)env * N + lane;
        if constexpr (MODE == kTdm)
          bot_combat_row(obs + row * (N - 1) * 4, TB.mask_out + row * (N - 1), N, pol_out + row * 4);
        else
          bot_flock_row(obs + row * od, (int)od, pol_out + row * 3);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __syncthreads();
    }
  }
  if constexpr (MODE == kTdm) {
    if (tl.ctl) {  // the tail observation: publish the last step, then observe rows until none is left
      if (phys) {
        __builtin_amdgcn_s_waitcnt(0);
        if (threadIdx.x == 0)
          __hip_atomic_store(tl.ctl + 2 * kTailQ * kTailLine + env, ((unsigned long long)tl.tag << 32) | (unsigned)tl.nsteps,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (blockIdx.x == 0 && threadIdx.x < kTailQ)  // the next launch's row counters (not this launch's)
        __hip_atomic_store(tl.ctl + (size_t)((((tl.tag + 1u) & 1u) * kTailQ + threadIdx.x) * kTailLine), 0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tl.worker = true;
      tl.k = A0.tail_k0;  // the worker's row offset: tail step k is launch step k0 + k
      int sl = (int)threadIdx.x;
      asm volatile("" : "+v"(sl));
      while (tl.more)
        step_w64_body<MODE, NCAP, OT, SCAL>(A0.P, A0.B, A0.TP, A0.TB, A0.cur, nullptr, A0.obs, nullptr, nullptr, nullptr,
                                            nullptr, env, sl, &tl);
    }
  }
}

// Resident blocks of the TDM rollout kernel on this device (the tail observation needs every block
// of a launch resident at once: a worker waits for envs whose waves must be running)
int tdm_rollout_resident_blocks(int n_agents, bool obs_f64) {
  const void* k = n_agents <= 32 ? (obs_f64 ? (const void*)env_rollout_w64<kTdm, 32, double>
                                            : (const void*)env_rollout_w64<kTdm, 32, float>)
                                 : (obs_f64 ? (const void*)env_rollout_w64<kTdm, 64, double>
                                            : (const void*)env_rollout_w64<kTdm, 64, float>);
  int per = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, W, 0) != hipSuccess || hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return per * cus;
}

template <int MODE, int NCAP, typename OT, bool SCAL = false>
static void launch_roll(int nsteps, unsigned long long astride, int traj, hipStream_t s, const StepParams& P,
                        const WorldBuffers& B, const TdmParams& TP, const TdmBuffers& TB, int cur, const void* actions,
                        void* obs, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done,
                        unsigned long long* tail_ctl = nullptr, unsigned tail_tag = 0u, int tail_workers = 0,
                        int tail_k0 = 0) {
  // astride == 0: closed loop, `actions` is the bots' action buffer (macm_world_rollout_bots)
  uint8_t* pol = astride == 0 ? static_cast<uint8_t*>(const_cast<void*>(actions)) : nullptr;
  const bool bal = B.sched && nsteps >= kRollBalanceMinSteps;
  if (bal) {
    // list sizes above kSchedMaxSize share the top bucket (any order among them is a valid order;
    // the histogram stays within 16 KB of LDS whatever max_contacts a world was given)
    const int CB = P.max_contacts < kSchedMaxSize ? P.max_contacts : kSchedMaxSize;
    hipLaunchKernelGGL(rollout_sched, dim3(1), dim3(1024), sizeof(uint32_t) * (CB + 1), s,
                       reinterpret_cast<const uint32_t*>(B.ccount[cur]), B.sched, P.n_envs, CB, nullptr);
    if (hipPeekAtLastError() != hipSuccess) return;  // no rollout on a stale order (the caller reports it)
  }
  RolloutArgs<OT> A{P, B, TP, TB, actions, (OT*)obs, nbr, rew, coll, done, astride, cur, nsteps, pol, traj, 0,
                    tail_ctl, tail_tag, tail_tag ? tail_k0 : 0};
  const int blocks = P.n_envs + (tail_tag ? tail_workers : 0);
  hipLaunchKernelGGL((env_rollout_w64<MODE, NCAP, OT, SCAL>), dim3(blocks), dim3(W), 0, s, A);
}

// the same instantiation choice as launch_step_w64 / launch_tdm_step_w64
// order[0..E): the envs by descending contact-list size (the workgroup step, kWgEnvOrder)
hipError_t launch_env_order(const uint32_t* ccount, uint32_t* order, int E, int C, hipStream_t s, unsigned int* reset2) {
  const int CB = C < kSchedMaxSize ? C : kSchedMaxSize;
  hipLaunchKernelGGL(rollout_sched, dim3(1), dim3(1024), sizeof(uint32_t) * (CB + 1), s, ccount, order, E, CB, reset2);
  return hipGetLastError();
}

hipError_t launch_rollout_w64(const StepParams& P, const WorldBuffers& B, int cur, const void* actions, void* obs,
                              bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done, hipStream_t s,
                              int nsteps, unsigned long long astride, int traj) {
  const TdmParams TP{};
  const TdmBuffers TB{};
  const bool small = P.n_agents <= 32;
  if (obs_f64) {
    if (small)
      launch_roll<kFlock, 32, double>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
    else
      launch_roll<kFlock, 64, double>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
  } else {
    if (small)
      launch_roll<kFlock, 32, float>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
    else if (P.n_envs >= kScalarSweepMinEnvs)
      launch_roll<kFlock, 64, float, true>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll,
                                           done);
    else
      launch_roll<kFlock, 64, float>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
  }
  return hipGetLastError();
}

hipError_t launch_tdm_rollout_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                                  const TdmBuffers& TB, int cur, const void* actions, void* obs, bool obs_f64,
                                  uint8_t* done, hipStream_t s, int nsteps, unsigned long long astride, int traj,
                                  unsigned long long* tail_ctl, unsigned tail_tag, int tail_workers,
                                  int tail_k0) {
  const bool small = P.n_agents <= 32;
  if (obs_f64) {
    if (small)
      launch_roll<kTdm, 32, double>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr,
                                    nullptr, done, tail_ctl, tail_tag, tail_workers, tail_k0);
    else
      launch_roll<kTdm, 64, double>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr,
                                    nullptr, done, tail_ctl, tail_tag, tail_workers, tail_k0);
  } else {
    if (small)
      launch_roll<kTdm, 32, float>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr,
                                   nullptr, done, tail_ctl, tail_tag, tail_workers, tail_k0);
    else
      launch_roll<kTdm, 64, float>(nsteps, astride, traj, s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr,
                                   nullptr, done, tail_ctl, tail_tag, tail_workers, tail_k0);
  }
  return hipGetLastError();
}

#else  // the one-step kernels, reset / observe kernels and their launchers
template <int MODE, int NCAP, typename OT, bool SCAL = false>
__global__ __launch_bounds__(W) __attribute__((amdgpu_waves_per_eu(4))) void env_step_w64(
    StepParams P, WorldBuffers B, TdmParams TP, TdmBuffers TB, int cur, const void* __restrict__ actions,
    OT* __restrict__ obs, int32_t* __restrict__ nbr_out, float* __restrict__ rew_out,
    uint8_t* __restrict__ coll_out, uint8_t* __restrict__ done_out) {
  step_w64_body<MODE, NCAP, OT, SCAL>(P, B, TP, TB, cur, actions, obs, nbr_out, rew_out, coll_out, done_out);
}

// Initial proxies (b2DynamicTree::CreateProxy: fat = tight +- 0.1), the first
// FindNewContacts' list (all overlapping pairs, descending), zeroed dynamics,
// and the initial observation (Flock.obs, mvmnt.py:79).
template <typename OT>
__global__ __launch_bounds__(W) void flock_init_w64(StepParams P, WorldBuffers B, int cur,
                                                    OT* __restrict__ obs, int32_t* __restrict__ nbr_out,
                                                    const uint8_t* __restrict__ mask) {
  const int e = blockIdx.x;
  if (mask && !mask[e]) return;  // reset_envs: only the masked envs
  const int lane = threadIdx.x;
  const int N = P.n_agents;
  const int C = P.max_contacts;
  const bool act = lane < N;
  const size_t ag = (size_t)e * N + lane;
  float2 p = make_float2(0.0f, 0.0f);
  float4 f = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float ang = 0.0f;
  float2 tg = make_float2(0.0f, 0.0f);
  if (act) {
    p = B.pos[ag];
    ang = B.angle[ag];
    tg = B.targets[(size_t)e * P.n_targets + B.tidx[lane]];
    const float r = P.radius;
    f = make_float4((p.x - r) - kAabbExtension, (p.y - r) - kAabbExtension, (p.x + r) + kAabbExtension,
                    (p.y + r) + kAabbExtension);
    B.fat[ag] = f;
    B.vel[ag] = make_float2(0.0f, 0.0f);
    B.sleep[ag] = 0.0f;
  }
  unsigned long long m = 0ull;
  float best = __builtin_inff();
  int bj = lane == 0 ? 1 : 0;
  for (int j = 0; j < N; ++j) {
    const float4 fj = make_float4(bcast(f.x, j), bcast(f.y, j), bcast(f.z, j), bcast(f.w, j));
    const float dx = bcast(p.x, j) - p.x, dy = bcast(p.y, j) - p.y;
    const float d2 = dx * dx + dy * dy;
    if (j > lane && overlap(f, fj)) m |= 1ull << j;
    if (j != lane && d2 < best) {
      best = d2;
      bj = j;
    }
  }
  int total = write_new_pairs(lane, act ? m : 0ull, B.cab[cur] + (size_t)e * C, B.cimp[cur] + (size_t)e * C, C);
  int st = 0;
  if (total > C) {
    st = MACM_ST_CONTACT_OVERFLOW;
    total = C;
  }
  const float bx = __shfl(p.x, bj, W), by = __shfl(p.y, bj, W);
  if (act) {
    if (nbr_out) nbr_out[ag] = bj;
    if (obs) {
      const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
      const float tdx = tg.x - p.x, tdy = tg.y - p.y;
      write_obs<OT>(obs + ag * od, P.coord, ang, best, bx - p.x, by - p.y, tdx, tdy, tdx * tdx + tdy * tdy);
    }
  }
  if (lane == 0) {
    B.ccount[cur][e] = total;
    B.step_count[e] = 0;
    B.time_passed[e] = 0.0;
    B.done[e] = 0;
    B.status[e] = st;
    if (st) report_status(B, st);
  }
}

// Observation of the current state (Flock.get_obs) without stepping.
template <typename OT>
__global__ __launch_bounds__(W) void flock_observe_w64(StepParams P, WorldBuffers B, OT* __restrict__ obs,
                                                       int32_t* __restrict__ nbr_out) {
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = P.n_agents;
  const bool act = lane < N;
  const size_t ag = (size_t)e * N + lane;
  float2 p = make_float2(0.0f, 0.0f), tg = make_float2(0.0f, 0.0f);
  float ang = 0.0f;
  if (act) {
    p = B.pos[ag];
    ang = B.angle[ag];
    tg = B.targets[(size_t)e * P.n_targets + B.tidx[lane]];
  }
  float best = __builtin_inff();
  int bj = lane == 0 ? 1 : 0;
  for (int j = 0; j < N; ++j) {
    const float dx = bcast(p.x, j) - p.x, dy = bcast(p.y, j) - p.y;
    const float d2 = dx * dx + dy * dy;
    if (j != lane && d2 < best) {
      best = d2;
      bj = j;
    }
  }
  const float bx = __shfl(p.x, bj, W), by = __shfl(p.y, bj, W);
  if (!act) return;
  if (nbr_out) nbr_out[ag] = bj;
  if (obs) {
    const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
    const float tdx = tg.x - p.x, tdy = tg.y - p.y;
    write_obs<OT>(obs + ag * od, P.coord, ang, best, bx - p.x, by - p.y, tdx, tdy, tdx * tdx + tdy * tdy);
  }
}

// TDM world creation (combat.py:78-101): every body active with init_health, zero
// cooldowns, the fresh listener, initial proxies / pairs as flock_init_w64, and
// the initial observation (self.obs = self.get_obs(), combat.py:102).
template <typename OT>
__global__ __launch_bounds__(W) void tdm_init_w64(StepParams P, WorldBuffers B, TdmParams TP, TdmBuffers TB,
                                                  int cur, OT* __restrict__ obs, const uint8_t* __restrict__ mask) {
  const int e = blockIdx.x;
  if (mask && !mask[e]) return;  // reset_envs: only the masked envs
  const int lane = threadIdx.x;
  const int N = P.n_agents;
  const int C = P.max_contacts;
  const bool act = lane < N;
  const size_t ag = (size_t)e * N + lane;
  __shared__ float2 s_p[W];
  __shared__ float s_a[W];
  float2 p = make_float2(0.0f, 0.0f);
  float4 f = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float ang = 0.0f;
  if (act) {
    p = B.pos[ag];
    ang = B.angle[ag];
    const float r = P.radius;
    f = make_float4((p.x - r) - kAabbExtension, (p.y - r) - kAabbExtension, (p.x + r) + kAabbExtension,
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
  }
  unsigned long long m = 0ull;
  for (int j = 0; j < N; ++j) {
    const float4 fj = make_float4(bcast(f.x, j), bcast(f.y, j), bcast(f.z, j), bcast(f.w, j));
    if (j > lane && overlap(f, fj)) m |= 1ull << j;
  }
  int total = write_new_pairs(lane, act ? m : 0ull, B.cab[cur] + (size_t)e * C, B.cimp[cur] + (size_t)e * C, C);
  int st = 0;
  if (total > C) {
    st = MACM_ST_CONTACT_OVERFLOW;
    total = C;
  }
  s_p[lane] = p;
  s_a[lane] = ang;
  const unsigned long long livem = __ballot(act);
  __syncthreads();
  const size_t rows = (size_t)e * N * (N - 1);
  tdm_obs_pairs<OT>(obs ? obs + rows * 4 : nullptr, TB.mask_out ? TB.mask_out + rows : nullptr, N, lane, livem, TP,
                   s_p, s_a);
  if (lane == 0) {
    B.ccount[cur][e] = total;
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

// TDM.get_obs of the current state without stepping.
template <typename OT>
__global__ __launch_bounds__(W) void tdm_observe_w64(StepParams P, WorldBuffers B, TdmParams TP, TdmBuffers TB,
                                                     OT* __restrict__ obs) {
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = P.n_agents;
  const size_t ag = (size_t)e * N + lane;
  __shared__ float2 s_p[W];
  __shared__ float s_a[W];
  bool live = false;
  if (lane < N) {
    const float2 p = B.pos[ag];
    s_p[lane] = p;
    s_a[lane] = B.angle[ag];
    live = TB.alive[ag] != 0;
  }
  const unsigned long long livem = __ballot(live);
  __syncthreads();
  const size_t rows = (size_t)e * N * (N - 1);
  tdm_obs_pairs<OT>(obs ? obs + rows * 4 : nullptr, TB.mask_out ? TB.mask_out + rows : nullptr, N, lane, livem, TP,
                   s_p, s_a);
}

// ---- host-side launchers (C++ linkage, used by macm_capi.hip) -----------------
template <int MODE, int NCAP, typename OT, bool SCAL = false>
static void launch_w64(hipStream_t s, const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                       const TdmBuffers& TB, int cur, const void* actions, void* obs, int32_t* nbr, float* rew,
                       uint8_t* coll, uint8_t* done) {
  hipLaunchKernelGGL((env_step_w64<MODE, NCAP, OT, SCAL>), dim3(P.n_envs), dim3(W), 0, s, P, B, TP, TB, cur, actions,
                     (OT*)obs, nbr, rew, coll, done);
}

hipError_t launch_step_w64(const StepParams& P, const WorldBuffers& B, int cur, const void* actions,
                           void* obs, bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done,
                           hipStream_t s) {
  const TdmParams TP{};
  const TdmBuffers TB{};
  const bool small = P.n_agents <= 32;
  if (obs_f64) {
    if (small)
      launch_w64<kFlock, 32, double>(s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
    else
      launch_w64<kFlock, 64, double>(s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
  } else {
    if (small)
      launch_w64<kFlock, 32, float>(s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
    else if (P.n_envs >= kScalarSweepMinEnvs)
      launch_w64<kFlock, 64, float, true>(s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
    else
      launch_w64<kFlock, 64, float>(s, P, B, TP, TB, cur, actions, obs, nbr, rew, coll, done);
  }
  return hipGetLastError();
}

hipError_t launch_tdm_step_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                               const TdmBuffers& TB, int cur, const void* actions, void* obs, bool obs_f64,
                               uint8_t* done, hipStream_t s) {
  const bool small = P.n_agents <= 32;
  if (obs_f64) {
    if (small)
      launch_w64<kTdm, 32, double>(s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr, nullptr, done);
    else
      launch_w64<kTdm, 64, double>(s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr, nullptr, done);
  } else {
    if (small)
      launch_w64<kTdm, 32, float>(s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr, nullptr, done);
    else
      launch_w64<kTdm, 64, float>(s, P, B, TP, TB, cur, actions, obs, nullptr, nullptr, nullptr, done);
  }
  return hipGetLastError();
}

hipError_t launch_tdm_init_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                               const TdmBuffers& TB, int cur, void* obs, bool obs_f64, const uint8_t* mask,
                               hipStream_t s) {
  dim3 grid(P.n_envs), block(W);
  if (obs_f64)
    hipLaunchKernelGGL(tdm_init_w64<double>, grid, block, 0, s, P, B, TP, TB, cur, (double*)obs, mask);
  else
    hipLaunchKernelGGL(tdm_init_w64<float>, grid, block, 0, s, P, B, TP, TB, cur, (float*)obs, mask);
  return hipGetLastError();
}

hipError_t launch_tdm_observe_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                                  const TdmBuffers& TB, void* obs, bool obs_f64, hipStream_t s) {
  dim3 grid(P.n_envs), block(W);
  if (obs_f64)
    hipLaunchKernelGGL(tdm_observe_w64<double>, grid, block, 0, s, P, B, TP, TB, (double*)obs);
  else
    hipLaunchKernelGGL(tdm_observe_w64<float>, grid, block, 0, s, P, B, TP, TB, (float*)obs);
  return hipGetLastError();
}

hipError_t launch_init_w64(const StepParams& P, const WorldBuffers& B, int cur, void* obs, bool obs_f64,
                           int32_t* nbr, const uint8_t* mask, hipStream_t s) {
  dim3 grid(P.n_envs), block(W);
  if (obs_f64)
    hipLaunchKernelGGL(flock_init_w64<double>, grid, block, 0, s, P, B, cur, (double*)obs, nbr, mask);
  else
    hipLaunchKernelGGL(flock_init_w64<float>, grid, block, 0, s, P, B, cur, (float*)obs, nbr, mask);
  return hipGetLastError();
}

hipError_t launch_observe_w64(const StepParams& P, const WorldBuffers& B, void* obs, bool obs_f64, int32_t* nbr,
                              hipStream_t s) {
  dim3 grid(P.n_envs), block(W);
  if (obs_f64)
    hipLaunchKernelGGL(flock_observe_w64<double>, grid, block, 0, s, P, B, (double*)obs, nbr);
  else
    hipLaunchKernelGGL(flock_observe_w64<float>, grid, block, 0, s, P, B, (float*)obs, nbr);
  return hipGetLastError();
}

#endif  // MACM_ROLLOUT_TU

}  // namespace macm
