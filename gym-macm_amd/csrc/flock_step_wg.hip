// flock_step_wg.hip — batched Flock env.step for 64 < N <= 1024 agents per env.
//
// Same algorithm and Box2D-order representation as flock_step_w64.hip (read its
// header first); this variant runs ONE WORKGROUP per env with one agent per
// thread (blockDim = N rounded up to 64, up to 1024 = 16 waves) and block-level
// primitives in place of single-wave ones:
//   * ordered compaction of the contact list by block-wide scans;
//   * touching edges as CSR (counts -> scan -> LDS-atomic fill -> per-body
//     insertion sort back into list order), no per-body degree cap;
//   * island DFS in Box2D order: sparse worlds find the islands first (union-find)
//     and walk them one thread per island, dense ones walk a popped body's edges
//     wave-parallel; the touching contacts are then written in Gauss-Seidel level
//     order for the solver;
//   * all-pairs sweep over per-agent records in LDS (broadcast reads); new
//     contacts = Ov(F_t) \ Ov(F_{t-1}) by testing the old fat AABBs, counted per
//     agent then written in descending (a, b) order after a descending scan.
// The step is split in three launches (kernels A, B, C below). An env whose touching
// contacts exceed kernel A's LDS capacity is stepped whole by the spill step
// (flock_spill.hpp) inside kernel A, and B and C skip it.
#include <map>
#include <type_traits>
#include <mutex>

#include "bots.hpp"
#include "flock_common.hpp"
#include "flock_spill.hpp"
#include "flock_grid.hpp"

namespace macm {
hipError_t launch_env_order(const uint32_t* ccount, uint32_t* order, int E, int C, hipStream_t s,
                            unsigned int* reset2 = nullptr);

// The step's env order (round 4): before each step the envs are ordered by contact-list size,
// heaviest first (launch_env_order, one workgroup), and workgroup b of kernels A, DFS, B and C
// steps env order[b]. Kernels A and C take several dispatch rounds (more workgroups than fit the
// chip at once), so the heaviest envs start in the first round instead of ending a late one, and
// kernel B's heaviest waves start one per SIMD. Any order gives the same results: every env is
// stepped by exactly one workgroup of each kernel.
__device__ __forceinline__ int wg_env(const WorldBuffers& B) {
  return B.sched ? (int)B.sched[blockIdx.x] : (int)blockIdx.x;
}

// ---- the B -> C handoff (flock_common.hpp Handoff) -------------------------------------------------
// Kernel B: every wave adds itself to b_started at its start (the second stream's wait), and
// publishes its env when its body ends, whichever return it takes (the guard's destructor): its
// stores of what C reads were write-through (st_wt: x_vout, x_cout, x_isolv, the list-order
// impulses), all its stores complete (vmcnt 0), then the env at the next slot of the finish order
// (an agent-scope atomic and an sc1 store; kernel C's block may run on another XCD).
struct HandoffPublish {
  const Handoff& H;
  int e;
  __device__ HandoffPublish(const Handoff& h, int env) : H(h), e(env) {
    if (H.q && threadIdx.x == 0) __hip_atomic_fetch_add(H.b_started, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ ~HandoffPublish() {
    if (!H.q) return;
    __builtin_amdgcn_s_waitcnt(0);
    if (threadIdx.x == 0) {
      const unsigned slot = __hip_atomic_fetch_add(&H.ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&H.q[slot], ((unsigned long long)H.tag << 32) | (unsigned)e, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
};

// Kernel C: the block's env, the next one kernel B finished (thread 0 polls with sc1 loads; the other
// waves load after the barrier; every load of B's handed-off bytes is ld_wt). A wait of ~1 s (never
// expected: every B wave is running when C is launched and waits for nothing) gives up:
// MACM_ST_HANDOFF, the block steps nothing (returns -1).
constexpr unsigned kHandoffSpins = 1u << 21;
__device__ __forceinline__ int handoff_take(const WorldBuffers& B, const Handoff& H, int* s_env) {
  if (threadIdx.x == 0) {
    const unsigned idx = __hip_atomic_fetch_add(&H.ctr[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int env = -1;
    for (unsigned it = 0; it < kHandoffSpins; ++it) {
      const unsigned long long v = __hip_atomic_load(&H.q[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((unsigned)(v >> 32) == H.tag) {
        env = (int)(unsigned)v;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (env < 0) report_status(B, MACM_ST_HANDOFF);
    *s_env = env;
  }
  __syncthreads();
  const int env = *s_env;
  __syncthreads();  // every thread has read it before the kernel reuses the word
  return env;
}

// The dependency the handoff needs is "every wave of kernel B has started", which no stream or event
// expresses (an event completes with a kernel). hipStreamWaitValue64 does (the first form), but each
// wait cost ~1 ms of latency on the MI355X (C3, 1000 envs: 281 -> 1,360 us per step). This watcher,
// one wave launched ahead of the consumer on its stream, polls the count (agent-scope loads) and
// ends as soon as it reaches `target`; the consumer is launched after it. It takes one wave slot and
// no LDS, so the producer's waves always fit beside it. A wait of ~1 s (never expected) reports
// MACM_ST_HANDOFF and ends.
constexpr unsigned kWatchSpins = 1u << 22;
__global__ __launch_bounds__(64) void wait_count(const unsigned long long* __restrict__ ctr, unsigned long long target,
                                                uint32_t* host_status) {
  if (threadIdx.x != 0) return;
  for (unsigned it = 0; it < kWatchSpins; ++it) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
    __builtin_amdgcn_s_sleep(1);
  }
  if (host_status) __hip_atomic_store(host_status, (uint32_t)MACM_ST_HANDOFF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
hipError_t launch_wait_count(const unsigned long long* ctr, unsigned long long target, uint32_t* host_status,
                             hipStream_t s) {
  hipLaunchKernelGGL(wait_count, dim3(1), dim3(64), 0, s, ctr, target, host_status);
  return hipGetLastError();
}

namespace wg {

constexpr int W = 64;
constexpr int kNewSlots = 8;  // kernel C, all-pairs sweep: new partners kept per body (16 B of LDS)
// Kernel A's island DFS in sparse worlds (average touching degree < 4): the islands are found
// first (union-find over the touching contacts, in parallel), each gets its contact and body
// ranges from its size and seed order, and then one thread walks each island, all islands at
// once, with the serial walk's code: the same order, levels and records as one thread walking
// them all in turn. Islands of more than kBigIsland contacts get a whole wave each (the dense
// path's wave-parallel walk). The walks run at issue priority 3.
constexpr int kBigIsland = 48;
// Dense envs (the wave-parallel walk: average touching degree >= 4, e.g. C5) take the island DFS,
// the Gauss-Seidel levels and the level-ordered records in their own kernel (flock_dfs_wg: one wave
// per env, ~45 KB of LDS, so 3 envs share a CU), instead of in kernel A, whose 78 KB block would
// hold a CU while one of its 16 waves walks.
// Kernel B's issue priority by the env's Gauss-Seidel depth (round 4) was dropped with the packed
// level steps (round 5: C3 window -1.3 / -1.7%, C3 closed loop -1.9%, C5 even without it;
// profiles/r05/abtests/solve_priority).
constexpr int kDfsPending = -2;  // x_nisl: the env's DFS is flock_dfs_wg's
// Kernel B's level steps: the idle lanes share one dummy slot (an LDS broadcast; a slot per lane,
// round 3, was slower); their position minima keep a word each.
constexpr int kDfsBatch = 8;  // contacts per lane whose loads flock_dfs_wg's record pass issues together

// Diagnostic build only (-DMACM_STAMPS): thread 0 records s_memtime after the
// block barrier that closes each phase into B.stamps[e][0..12] (tools/phase_profile.py
// --kernel wg). The product library compiles these to nothing.
#ifdef MACM_STAMPS
#define WSTAMP(k)                                                       \
  do {                                                                  \
    __builtin_amdgcn_s_waitcnt(0);                                      \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();         \
    if (tid == 0) B.stamps[(size_t)e * 32 + (k)] = _t;                  \
  } while (0)
#else
#define WSTAMP(k) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ float bmin(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float bmax(float a, float b) { return a > b ? a : b; }
// The contact solvers' clamps as single v_min_f32 / v_max_f32 instead of compare + select
// (b2Min / b2Max): they sit on the serial Gauss-Seidel chain. For non-NaN operands the two
// forms differ only in the sign of a zero result (b2Max(-0, +0) is +0, v_max may give -0);
// a zero impulse or velocity of either sign leaves every later value the same, so only
// zero signs can differ (as they already do through the angular terms).
// sclamp as one v_med3_f32 (as in flock_step_w64.hip)
__device__ __forceinline__ float smax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ float sclamp(float a, float lo, float hi) { return __builtin_amdgcn_fmed3f(a, lo, hi); }
__device__ __forceinline__ bool overlap(float4 a, float4 b) {  // b2TestOverlap
  const float d1x = b.x - a.z, d1y = b.y - a.w;
  const float d2x = a.x - b.z, d2y = a.y - b.w;
  if (d1x > 0.0f || d1y > 0.0f) return false;
  if (d2x > 0.0f || d2y > 0.0f) return false;
  return true;
}
// max of the four AABB separations; > 0 iff b2TestOverlap(a, b) is false (finite boxes)
__device__ __forceinline__ float sep_max(float4 a, float4 b) {
  return fmaxf(fmaxf(b.x - a.z, b.y - a.w), fmaxf(a.x - b.z, a.y - b.w));
}
__device__ __forceinline__ void normalize(float& x, float& y) {  // b2Vec2::Normalize (see sqrt_rn / rcp_rn)
  const float len = sqrt_rn(x * x + y * y);
  if (len < kEps) return;
  const float inv = rcp_rn(len);
  x *= inv;
  y *= inv;
}

struct __align__(16) Rec {  // per-agent record for the pair sweep (48 B with float4 alignment)
  float4 fn;               // new fat AABB
  float4 fo;               // old fat AABB
  float2 c;                // final position
};


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

}  // namespace wg

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

// Reset for the workgroup variant: fat AABBs, first FindNewContacts list (all
// overlapping pairs, descending), zeroed dynamics, initial observation.
template <typename OT>
__global__ __launch_bounds__(1024) void flock_init_wg(StepParams P, WorldBuffers B, int cur, OT* __restrict__ obs,
                                                      int32_t* __restrict__ nbr_out,
                                                      const uint8_t* __restrict__ mask) {
  using namespace wg;
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x, tid = threadIdx.x, N = P.n_agents, C = P.max_contacts;
  if (mask && !mask[e]) return;  // reset_envs: only the masked envs (mask is not written here)
  const bool act = tid < N;
  const size_t ag = (size_t)e * N + tid;
  Rec* s_rec = (Rec*)lds;
  int* s_scan = (int*)(lds + align16((int)sizeof(Rec) * N));
  float2 p = make_float2(0.0f, 0.0f), tg = make_float2(0.0f, 0.0f);
  float ang = 0.0f;
  float4 f = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (act) {
    p = B.pos[ag];
    ang = B.angle[ag];
    tg = B.targets[(size_t)e * P.n_targets + B.tidx[tid]];
    const float r = P.radius;
    f = make_float4((p.x - r) - kAabbExtension, (p.y - r) - kAabbExtension, (p.x + r) + kAabbExtension,
                    (p.y + r) + kAabbExtension);
    B.fat[ag] = f;
    B.vel[ag] = make_float2(0.0f, 0.0f);
    B.sleep[ag] = 0.0f;
    Rec r0;
    r0.fn = f;
    r0.fo = f;
    r0.c = p;
    s_rec[tid] = r0;
  }
  __syncthreads();
  WSTAMP(9);
  int cnt = 0;
  float best = __builtin_inff();
  int bj = tid == 0 ? 1 : 0;
  if (act)
    for (int j = 0; j < N; ++j) {
      const Rec r = s_rec[j];
      if (j > tid && overlap(f, r.fn)) ++cnt;
      const float dx = r.c.x - p.x, dy = r.c.y - p.y;
      const float d2 = dx * dx + dy * dy;
      if (j != tid && d2 < best) {
        best = d2;
        bj = j;
      }
    }
  int excl;
  int total = block_scan_excl(cnt, excl, s_scan);
  if (act && cnt > 0) {
    int w = total - excl - cnt;
    for (int j = N - 1; j > tid; --j)
      if (overlap(f, s_rec[j].fn)) {
        if (w < C) {
          B.cab[cur][(size_t)e * C + w] = (uint32_t)tid | ((uint32_t)j << 16);
          B.cimp[cur][(size_t)e * C + w] = make_float2(0.0f, 0.0f);
        }
        ++w;
      }
  }
  if (act) {
    if (nbr_out) nbr_out[ag] = bj;
    if (obs) {
      const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
      const float tdx = tg.x - p.x, tdy = tg.y - p.y;
      const float2 cb = s_rec[bj].c;
      write_obs<OT>(obs + ag * od, P.coord, ang, best, cb.x - p.x, cb.y - p.y, tdx, tdy, tdx * tdx + tdy * tdy);
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

template <typename OT>
__global__ __launch_bounds__(1024) void flock_observe_wg(StepParams P, WorldBuffers B, OT* __restrict__ obs,
                                                         int32_t* __restrict__ nbr_out) {
  using namespace wg;
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x, tid = threadIdx.x, N = P.n_agents;
  const bool act = tid < N;
  const size_t ag = (size_t)e * N + tid;
  float2* s_p = (float2*)lds;
  float2 p = make_float2(0.0f, 0.0f);
  if (act) {
    p = B.pos[ag];
    s_p[tid] = p;
  }
  __syncthreads();
  if (!act) return;
  float best = __builtin_inff();
  int bj = tid == 0 ? 1 : 0;
  for (int j = 0; j < N; ++j) {
    const float2 q = s_p[j];
    const float dx = q.x - p.x, dy = q.y - p.y;
    const float d2 = dx * dx + dy * dy;
    if (j != tid && d2 < best) {
      best = d2;
      bj = j;
    }
  }
  if (nbr_out) nbr_out[ag] = bj;
  if (obs) {
    const float2 tg = B.targets[(size_t)e * P.n_targets + B.tidx[tid]];
    const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
    const float tdx = tg.x - p.x, tdy = tg.y - p.y;
    write_obs<OT>(obs + ag * od, P.coord, B.angle[ag], best, s_p[bj].x - p.x, s_p[bj].y - p.y, tdx, tdy,
                  tdx * tdx + tdy * tdy);
  }
}

// ==== split step for large N =========================================================================
// A single fused kernel would keep one env's whole world in LDS (up to ~134 KB at N = 1024), so a
// CU would hold one env, and while that env's single Gauss-Seidel lane walks a dense island the
// rest of the CU would idle (measured 72.6 ms vs 18.2 ms per C5 step in round 1). The step runs
// as three launches:
//   A  flock_step_wg_a : actions, Collide, CSR edges, island DFS, velocity integration, and the
//                        island-ordered contact records written to HBM (x_cst / x_cimp). Envs
//                        with more than tcap touching contacts take the spill step here instead
//                        (x_nisl = -1 tells B and C to skip them).
//   B  flock_solve_wg  : one wave per env, LDS = positions + velocities only (16 B per body):
//                        warm start, velocity iterations, StoreImpulses, position integration,
//                        position iterations. Contacts stream from HBM two records ahead
//                        (islands of >= 3 contacts; smaller islands stay in registers).
//   C  flock_step_wg_c : sleep, SynchronizeFixtures, pair sweep, next contact list, rewards, obs,
//                        write-back.
// Every arithmetic operation and its order are those of the wave kernel and the spill step.

// Up to this many agents kernel A keeps each CSR edge's other body next to it (s_oth, 4 B per
// touching contact), so an island walk reads an edge and its other body in one LDS round trip
// instead of two (edge, then the contact's pair). Above it (78 KB of LDS at N = 1024, two blocks
// per CU) the walks read the pair.
constexpr int kOthMaxAgents = 512;
struct WgLayoutA {
  int c, deg, csr_off, todo, ord, ib, ibod, stk, ic, scan, misc, tab, adj, oth, total;
};
__host__ __device__ inline WgLayoutA wg_layout_a(int N, int tcap) {
  WgLayoutA L;
  int o = 0;
  auto take = [&](int bytes) {
    int r = o;
    o = align16(o + bytes);
    return r;
  };
  L.c = take(8 * N);
  L.deg = take(2 * (N + 2));
  L.csr_off = take(2 * (N + 1));
  L.todo = take(8 * ((N + 63) / 64));
  L.ord = take(2 * tcap);
  L.ib = take(2 * (N / 2 + 2));
  L.ibod = take(2 * N);
  L.stk = take(2 * (N + 16));  // the walks' stacks, then a dummy slot per wave
  L.ic = take(2 * (N / 2 + 2));
  L.scan = take(4 * 32);
  L.misc = take(4 * 8);
  L.tab = take(4 * tcap);
  L.adj = take(6 * tcap + 8);  // CSR edges (2 tcap u16), then level counts (tcap + 1 u32); levels (tcap u16) at 4 tcap + 8
  L.oth = N <= kOthMaxAgents ? take(4 * tcap) : -1;  // [2 tcap] the other body of CSR edge q
  L.total = o;
  return L;
}

struct WgLayoutC {
  int slp, flags, oldc, scan, misc, fn, fo, c, gred, gpar, gstart, gsext, gent, pk, bjv, total;
};
__host__ __device__ inline WgLayoutC wg_layout_c(int N) {
  WgLayoutC L;
  int o = 0;
  auto take = [&](int bytes) {
    int r = o;
    o = align16(o + bytes);
    return r;
  };
  L.slp = take(4 * N);
  L.flags = take(N);
  L.oldc = take(4 * ((N + 31) / 32));
  L.scan = take(4 * 32);
  L.misc = take(4 * 8);
  L.fn = take(16 * N);  // pair-sweep records, SoA: new fat AABB, old fat AABB, final position
  L.fo = take(16 * N);
  L.c = take(8 * N);
  L.gred = take(4 * 4 * 16);
  L.gpar = take(4 * 8);
  L.gstart = take(4 * (grid::buckets(N) + 1) > 2 * N + 4 ? 4 * (grid::buckets(N) + 1) : 2 * N + 4);
  L.gsext = take(4 * grid::buckets(N));
  L.gent = take(16 * N);
  L.pk = take(4 * N);   // per body: collided bit 31 | new-pair count (sweep)
  L.bjv = take(2 * N);  // per body: nearest neighbour (sweep); then new-pair segment starts
  L.total = o;
  return L;
}

__host__ __device__ inline int wg_isl_stride(int N) { return N / 2 + 2; }
// solver LDS: velocities + positions (16 B per body), record/impulse/ab rings, big-island list
// kernel B: velocities and positions (16 B per body), the islands' pass minima (which double as the
// velocity passes' 64 dummy slots, so at least 512 B), their solved flags, slack
__host__ __device__ inline int wg_solve_mins_bytes(int N) {
  return 4 * wg_isl_stride(N) > 512 ? 4 * wg_isl_stride(N) : 512;
}
__host__ __device__ inline int wg_solve_lds(int N) { return 16 * N + wg_solve_mins_bytes(N) + wg_isl_stride(N) + 16; }

template <typename OT>
__global__ __launch_bounds__(1024) void flock_step_wg_a(StepParams P, WorldBuffers B, int cur, int tcap,
                                                        const void* __restrict__ actions, OT* __restrict__ obs,
                                                        int32_t* __restrict__ nbr_out, float* __restrict__ rew_out,
                                                        uint8_t* __restrict__ coll_out,
                                                        uint8_t* __restrict__ done_out) {
  using namespace wg;
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = wg_env(B);
  const int tid = threadIdx.x;
  const int BS = blockDim.x;
  const int N = P.n_agents;
  const int C = P.max_contacts;
  const bool act = tid < N;
  const size_t ag = (size_t)e * N + tid;
  const WgLayoutA L = wg_layout_a(N, tcap);
  float2* s_c = (float2*)(lds + L.c);
  uint16_t* s_deg = (uint16_t*)(lds + L.deg);
  uint16_t* s_off = (uint16_t*)(lds + L.csr_off);
  unsigned long long* s_todo = (unsigned long long*)(lds + L.todo);
  uint16_t* s_ord = (uint16_t*)(lds + L.ord);
  uint16_t* s_ib = (uint16_t*)(lds + L.ib);
  uint16_t* s_ibod = (uint16_t*)(lds + L.ibod);
  uint16_t* s_stk = (uint16_t*)(lds + L.stk);
  uint16_t* s_ic = (uint16_t*)(lds + L.ic);
  int* s_scan = (int*)(lds + L.scan);
  int* s_misc = (int*)(lds + L.misc);
  uint32_t* s_tab = (uint32_t*)(lds + L.tab);
  uint16_t* s_adj = (uint16_t*)(lds + L.adj);
  float2* g_lam = B.scratch + (size_t)e * tcap;

  const uint32_t* cab = B.cab[cur] + (size_t)e * C;
  const float2* cimp = B.cimp[cur] + (size_t)e * C;
  const int step_count = B.step_count[e];
  const int M = B.ccount[cur][e];
  float2 p = make_float2(0.0f, 0.0f), v = make_float2(0.0f, 0.0f);
  float ang = 0.0f;
  int a0 = 1, a1 = 1, a2 = 1;
  float ax = 0.0f, ay = 0.0f;
  if (act) {
    p = B.pos[ag];
    v = B.vel[ag];
    ang = B.angle[ag];
    if (P.action_mode == MACM_ACTION_DISCRETE) {
      const uint8_t* a = (const uint8_t*)actions + ag * 3;
      a0 = a[0]; a1 = a[1]; a2 = a[2];
    } else {
      const float2 c = ((const float2*)actions)[ag];
      ax = c.x; ay = c.y;
    }
    s_c[tid] = p;
  }
  for (int q = tid; q < N + 2; q += BS) s_deg[q] = 0;
  if (tid < 8) s_misc[tid] = 0;
  WSTAMP(16);

  // ---- actions -> angle, force (mvmnt.py:97-129) ---------------------------------
  float Fx = 0.0f, Fy = 0.0f;
  if (act) {
    if (P.action_mode == MACM_ACTION_DISCRETE) {
      float af = (float)((double)ang + ((double)(a2 - 1) * P.rot_step) * P.inv_hz);
      double ad = (double)af;
      if (fabs(ad) > M_PI) {
        af = (float)(ad - sgn(ad) * (2.0 * M_PI));
        ad = (double)af;
      }
      ang = af;
      const double cc = ((a0 != 1) && (a1 != 1)) ? P.diag_c : 1.0;
      const double k0 = (double)(a0 - 1), k1 = (double)(a1 - 1);
      double s0, c0, s1, c1;
      act_trig(af, &s0, &c0, &s1, &c1);
      Fx = (float)((c0 * k0 + c1 * k1) * cc * P.force);
      Fy = (float)((s0 * k0 + s1 * k1) * cc * P.force);
    } else {
      float x = ax, y = ay;
      if ((x * x + y * y) > 1.0f) {
        x = sqrtf(x * x / (x * x + y * y));
        y = sqrtf(y * y / (x * x + y * y));
      }
      Fx = x * P.force_f32;
      Fy = y * P.force_f32;
    }
    Fx = 0.0f + Fx;
    Fy = 0.0f + Fy;
  }
  __syncthreads();
  WSTAMP(17);

  // ---- Collide: ordered compaction of the touching contacts -----------------------
  const float rr = (P.radius + P.radius) * (P.radius + P.radius);
  const float dt_ratio = step_count > 0 ? P.inv_dt * P.dt : 0.0f;
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
      const float2 pa = s_c[a], pb = s_c[b];
      const float dx = pb.x - pa.x, dy = pb.y - pa.y;
      touch = !(dx * dx + dy * dy > rr);  // b2CollideCircles
    }
    int pos;
    const int n = block_scan_excl(touch ? 1 : 0, pos, s_scan);
    if (touch && T + pos < tcap) {
      s_tab[T + pos] = ab;
      g_lam[T + pos] = P.warm_starting ? make_float2(dt_ratio * lam.x, dt_ratio * lam.y) : make_float2(0.0f, 0.0f);
    }
    T += n;
  }
  if (T > tcap || P.force_spill) {
    // More touching contacts than this kernel's LDS holds: the env's whole step runs here as the
    // spill step (HBM working set, flock_spill.hpp) from its untouched start-of-step state (only
    // scratch has been written so far), and kernels B and C skip it.
    spill::step_env<OT, false, kFlock, 1, true>(P, B, e, cur, actions, obs, nbr_out, rew_out, coll_out, done_out, lds);
    if (tid == 0) B.x_nisl[e] = -1;
    return;
  }
  if (act) B.angle[ag] = ang;  // kernel C reads it for the observation
  __syncthreads();
  WSTAMP(18);

  // ---- CSR touching edges, each body's segment in list (= Box2D edge) order ---------
#define DEG_WORD(i) ((unsigned int*)(s_deg + ((i) & ~1)))
#define DEG_INC(i) (((i) & 1) ? 0x10000u : 1u)
#define DEG_GET(w, i) (((i) & 1) ? ((w) >> 16) : ((w) & 0xffffu))
  for (int t = tid; t < T; t += BS) {
    const uint32_t ab = s_tab[t];
    const int a = ab & 0xffffu, b = ab >> 16;
    atomicAdd(DEG_WORD(a), DEG_INC(a));
    atomicAdd(DEG_WORD(b), DEG_INC(b));
  }
  __syncthreads();
  const int deg = act ? (int)s_deg[tid] : 0;
  {
    int off;
    block_scan_excl(deg, off, s_scan);
    if (act) s_off[tid] = (uint16_t)off;
    if (tid == 0) s_off[N] = (uint16_t)(2 * T);
    const unsigned long long m = __ballot(act && deg > 0);
    if ((tid & (W - 1)) == 0 && tid / W < (N + 63) / 64) s_todo[tid / W] = m;
  }
  __syncthreads();
  if (act) s_deg[tid] = s_off[tid];
  __syncthreads();
  for (int t = tid; t < T; t += BS) {
    const uint32_t ab = s_tab[t];
    const int a = ab & 0xffffu, b = ab >> 16;
    const unsigned wa = atomicAdd(DEG_WORD(a), DEG_INC(a));
    const unsigned wb = atomicAdd(DEG_WORD(b), DEG_INC(b));
    s_adj[DEG_GET(wa, a)] = (uint16_t)t;
    s_adj[DEG_GET(wb, b)] = (uint16_t)t;
  }
#undef DEG_WORD
#undef DEG_INC
#undef DEG_GET
  __syncthreads();
  // Gauss-Seidel levels are computed during the DFS (below): s_last[b] = 1 + level of the last
  // contact, in island order, that touches body b (0 = none). s_deg is free from here on.
  uint16_t* s_last = s_deg;
  uint16_t* s_lvl = (uint16_t*)(lds + L.adj + 4 * tcap + 8);  // [tcap] level of island-ordered contact k
  uint16_t* s_oth = L.oth >= 0 ? (uint16_t*)(lds + L.oth) : nullptr;
  if (act) s_last[tid] = 0;
  if (act && deg > 1) {
    const int o0 = s_off[tid];
    for (int x = o0 + 1; x < o0 + deg; ++x) {
      const uint16_t key = s_adj[x];
      int y = x - 1;
      while (y >= o0 && s_adj[y] > key) {
        s_adj[y + 1] = s_adj[y];
        --y;
      }
      s_adj[y + 1] = key;
    }
  }
  if (s_oth && act)
    for (int q = s_off[tid], q1 = q + deg; q < q1; ++q) {
      const uint32_t ab = s_tab[s_adj[q]];
      s_oth[q] = (uint16_t)((int)(ab & 0xffffu) == tid ? ab >> 16 : ab & 0xffffu);
    }
  __syncthreads();
  WSTAMP(19);

  // ---- island DFS in Box2D order (as in flock_step_wg) ---------------------------------
  const bool par_dfs = 2 * T >= 4 * N;
  if (par_dfs) {
    // the touching contacts, the CSR offsets and every edge with its other body to HBM; the
    // integrated velocities as after the walk; flock_dfs_wg does the rest of this kernel
    const int IS = wg_isl_stride(N);
    (void)IS;
    uint32_t* xt = B.x_tab + (size_t)e * tcap;
    for (int t = tid; t < T; t += BS) xt[t] = s_tab[t];
    if (act) {
      uint32_t* xa = B.x_adj + (size_t)e * 2 * tcap;
      const int o0 = s_off[tid], o1 = o0 + deg;
      for (int q = o0; q < o1; ++q) {
        const int t = s_adj[q];
        const uint32_t ab = s_tab[t];
        const int a = ab & 0xffffu, b = ab >> 16;
        xa[q] = (uint32_t)t | ((uint32_t)(a == tid ? b : a) << 16);
      }
      B.x_off[(size_t)e * (N + 1) + tid] = s_off[tid];
      const float vx = v.x + P.dt * (0.0f + P.inv_mass * Fx);
      const float vy = v.y + P.dt * (0.0f + P.inv_mass * Fy);
      B.x_vmid[ag] = make_float2(vx * P.damp, vy * P.damp);
      B.x_deg[ag] = deg > 0 ? 1 : 0;
    }
    if (tid == 0) {
      B.x_off[(size_t)e * (N + 1) + N] = (uint16_t)(2 * T);
      B.x_nisl[e] = kDfsPending;
    }
#ifdef MACM_STAMPS
    if (tid == 0)
      for (int k = 20; k <= 22; ++k) B.stamps[(size_t)e * 32 + k] = B.stamps[(size_t)e * 32 + 19];
#endif
    return;
  }
  // Walk state per body in s_last: bits 0..13 = 1 + the level of the last walked contact touching
  // it (levels <= tcap < 2^14), bit 15 = pushed, bit 14 = popped. One LDS read of an edge's other
  // body gives everything the edge needs: the contact was walked iff the other body was popped (the
  // first of its two bodies to be popped walks it), the body is pushed iff it was not pushed yet,
  // and the level chain's input. A new contact's other body is pushed by then either way, so the
  // walk writes its word as level | pushed; a pop ends with level | pushed | popped. An edge's other
  // body comes from s_oth (N <= kOthMaxAgents; one read next to the edge's own) or from the
  // contact's pair. No todo bits or visited flags are written.
  constexpr int kPushed = 0x8000, kPopped = 0x4000, kLvl = 0x3fff;
  auto edge_other = [&](auto HO, int q, int t, int bdy) -> int {
    if constexpr (decltype(HO)::value) {
      (void)t;
      (void)bdy;
      return s_oth[q];
    } else {
      (void)q;
      const uint32_t ab = s_tab[t];
      const int a = ab & 0xffffu;
      return a == bdy ? (int)(ab >> 16) : a;
    }
  };
  // One island walked by a whole wave from seed sd (never touched yet: level 0): a popped body's
  // edges one per lane, levels by a prefix maximum (below). Appends to s_ord / s_lvl at nord and
  // s_ibod at nb; the stack lives at s_stk[sbase...], the wave's dummy slot at s_stk[N + wave].
  // Every lane of the wave calls it.
  auto par_walk = [&](auto HO, int sd, int& nord, int& nb, int sbase, int& dmax) {
    const int lane = tid & (W - 1);
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint16_t* stk = s_stk + sbase;
    uint16_t* const dummy = s_stk + N + tid / W;
    // the body to pop next with its CSR range and level: the seed, then the last push of the
    // previous pop (in registers; its stack slot is dropped), else the stack's top
    int sp = 1;
    int top_b = sd, top_e0 = s_off[sd], top_e1 = s_off[sd + 1], top_last = 0;
    __builtin_amdgcn_wave_barrier();
    while (sp > 0) {
      int bdy, e0, e1, xcur;
      --sp;
      if (top_b >= 0) {
        bdy = top_b;
        e0 = top_e0;
        e1 = top_e1;
        xcur = top_last;
      } else {
        bdy = stk[sp];
        e0 = s_off[bdy];
        e1 = s_off[bdy + 1];
        xcur = s_last[bdy] & kLvl;
      }
      top_b = -1;
      if (lane == 0) s_ibod[nb] = (uint16_t)bdy;
      ++nb;
      // Levels of the new contacts c_1..c_m of bdy, in order (all touch bdy; their other bodies
      // o_i are distinct): with X_0 = last[bdy] and y_i = last[o_i], the serial rule
      // X_i = max(X_{i-1}, y_i) + 1 gives X_i = i + max(X_0, max_{j<=i}(y_j - j + 1)),
      // a prefix maximum over the lanes; level(c_i) = X_i - 1. Branch-free up to the stores:
      // lanes past the body's last edge read that edge and take no part.
      for (int q0 = e0; q0 < e1; q0 += W) {
        const int q = min(q0 + lane, e1 - 1);
        const int t = s_adj[q];
        const int o = edge_other(HO, q, t, bdy);
        const int so = s_last[o];
        const int oe0 = s_off[o], oe1 = s_off[o + 1];
        const bool newc = q0 + lane < e1 && !(so & kPopped);
        const bool push = newc && !(so & kPushed);
        const unsigned long long mc = __ballot(newc), mp = __ballot(push);
        const int rank = __popcll(mc & lt) + 1;
        const int z = wave_prefix_max(newc ? (so & kLvl) - rank + 1 : -0x3fffffff);
        const int xi = rank + max(xcur, z);
        if (newc) {
          s_last[o] = (uint16_t)(xi | kPushed);
          s_ord[nord + rank - 1] = (uint16_t)t;
          s_lvl[nord + rank - 1] = (uint16_t)(xi - 1);
          *(push ? stk + sp + __popcll(mp & lt) : dummy) = (uint16_t)o;
        }
        const int mnew = __popcll(mc);
        if (mnew) xcur = mnew + max(xcur, __builtin_amdgcn_readlane(z, W - 1));
        nord += mnew;
        sp += __popcll(mp);
        if (mp) {  // the new top: the highest pushing lane
          const int hl = 63 - __clzll(mp);
          top_b = __builtin_amdgcn_readlane(o, hl);
          top_e0 = __builtin_amdgcn_readlane(oe0, hl);
          top_e1 = __builtin_amdgcn_readlane(oe1, hl);
          top_last = __builtin_amdgcn_readlane(xi, hl);
        }
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) s_last[bdy] = (uint16_t)(xcur | kPushed | kPopped);
      dmax = max(dmax, xcur);
      __builtin_amdgcn_wave_barrier();
    }
  };
  // One island walked by one thread from seed sd (never touched yet), Box2D's serial order: per
  // new contact, level = max(last[body], last[other]); the popped body's last stays in a register.
  // Appends to s_ord / s_lvl at nord and s_ibod at nb; the stack lives at s_stk[nb at entry...].
  auto serial_walk = [&](auto HO, int sd, int& nord, int& nb, int& dmax) {
    const int sb = nb;
    int sp = sb + 1;  // the seed, popped from registers
    int top_b = sd, top_e0 = s_off[sd], top_e1 = s_off[sd + 1], top_lb = 0;
    while (sp > sb) {
      --sp;
      int b, e0, e1, lb;
      if (top_b >= 0) {
        b = top_b;
        e0 = top_e0;
        e1 = top_e1;
        lb = top_lb;
      } else {
        b = s_stk[sp];
        e0 = s_off[b];
        e1 = s_off[b + 1];
        lb = s_last[b] & kLvl;
      }
      top_b = -1;
      s_ibod[nb++] = (uint16_t)b;
      // the next edge and its other body are read one edge ahead (the edges are not written
      // during the walk): an edge then costs one dependent LDS round trip (its other body's word)
      int tn = 0, on = 0;
      if (e0 < e1) {
        tn = s_adj[e0];
        on = edge_other(HO, e0, tn, b);
      }
      for (int q = e0; q < e1; ++q) {
        const int t = tn, o = on;
        const int qn = min(q + 1, e1 - 1);
        tn = s_adj[qn];
        on = edge_other(HO, qn, tn, b);
        const int so = s_last[o];
        const int oe0 = s_off[o], oe1 = s_off[o + 1];
        if (so & kPopped) continue;
        const int l = max(lb, so & kLvl);  // level: 1 + the level of the last earlier contact touching b or o
        lb = l + 1;
        s_last[o] = (uint16_t)(lb | kPushed);
        s_lvl[nord] = (uint16_t)l;
        s_ord[nord++] = (uint16_t)t;
        if (so & kPushed) continue;
        s_stk[sp++] = (uint16_t)o;
        top_b = o;
        top_e0 = oe0;
        top_e1 = oe1;
        top_lb = lb;
      }
      s_last[b] = (uint16_t)(lb | kPushed | kPopped);
      dmax = max(dmax, lb);
    }
  };
#define MACM_WALK(f, ...) (s_oth ? f(std::true_type{}, __VA_ARGS__) : f(std::false_type{}, __VA_ARGS__))
  // Sparse worlds: islands first, then one thread per island (see kIslandDfs).
  const bool isl_dfs = !par_dfs && 2 * tcap >= 4 * N;
  if (isl_dfs) {
    // Union-find labels, hooking the lower root under the higher and jumping to the roots after
    // every round, so each component's root is its highest body: the seed the serial walk would
    // take (it seeds at the highest unvisited body with edges and consumes whole islands).
    uint32_t* s_lab = (uint32_t*)(lds + L.ord);  // [N]; s_ord is written only by the walks
    if (act) s_lab[tid] = (uint32_t)tid;
    __syncthreads();
#ifdef MACM_STAMPS
    const unsigned long long lab_t0 = __builtin_amdgcn_s_memtime();
    int lab_rounds = 0;
#endif
    for (;;) {
#ifdef MACM_STAMPS
      ++lab_rounds;
#endif
      bool hooked = false;
      for (int t = tid; t < T; t += BS) {
        const uint32_t ab = s_tab[t];
        const uint32_t ra = s_lab[ab & 0xffffu], rb = s_lab[ab >> 16];
        if (ra != rb) {
          hooked = true;
          if (ra < rb) atomicMax(&s_lab[ra], rb);
          else atomicMax(&s_lab[rb], ra);
        }
      }
      if (!__syncthreads_or(hooked)) break;
      if (act) {  // labels only grow along a chain, so the walk ends at the root
        uint32_t l = s_lab[tid], n;
        while ((n = s_lab[l]) != l) l = n;
        s_lab[tid] = l;
      }
      __syncthreads();
    }
#ifdef MACM_STAMPS
    if (tid == 0) {  // diagnostics: labeling cycles and rounds (tools/phase_profile.py)
      B.stamps[(size_t)e * 32 + 24] = __builtin_amdgcn_s_memtime() - lab_t0;
      B.stamps[(size_t)e * 32 + 25] = (unsigned long long)lab_rounds;
    }
#endif
    // islands in seed order = roots in descending order; rank per root in s_last (free until
    // the walks), island sizes (contacts | bodies << 16) in s_stk, island seeds in s_ibod
    uint32_t* s_isz = (uint32_t*)(lds + L.stk);
    uint16_t* s_seed = s_ibod;
    const bool root = act && deg > 0 && s_lab[tid] == (uint32_t)tid;
    int rexcl;
    const int nisl = block_scan_excl(root ? 1 : 0, rexcl, s_scan);
    if (tid < nisl) s_isz[tid] = 0u;
    if (root) {
      const int I = nisl - 1 - rexcl;
      s_last[tid] = (uint16_t)I;
      s_seed[I] = (uint16_t)tid;
    }
    __syncthreads();
    for (int t = tid; t < T; t += BS) atomicAdd(&s_isz[s_last[s_lab[s_tab[t] & 0xffffu]]], 1u);
    if (act && deg > 0) atomicAdd(&s_isz[s_last[s_lab[tid]]], 1u << 16);
    __syncthreads();
    const uint32_t sz = tid < nisl ? s_isz[tid] : 0u;
    const int seed = tid < nisl ? (int)s_seed[tid] : 0;
    int off;
    const int tot = block_scan_excl((int)sz, off, s_scan);  // contacts <= tcap, bodies <= N: no carry
    if (tid < nisl) {
      s_ic[tid] = (uint16_t)(off & 0xffff);
      s_ib[tid] = (uint16_t)(off >> 16);
    }
    if (tid == 0) {
      s_ic[nisl] = (uint16_t)(tot & 0xffff);
      s_ib[nisl] = (uint16_t)(tot >> 16);
      s_misc[0] = nisl;
    }
    if (act) s_last[tid] = 0;
    // Islands of more than kBigIsland contacts are walked by a whole wave each (par_walk), the
    // rest one per thread of the other waves. Work list (seed, contact | body offsets) in s_lab's
    // words (the labels are dead): the wave-walked islands first. nbw leaves a thread per island.
    const int nw = BS / W, wid = tid / W;
    const bool big = tid < nisl && (int)(sz & 0xffffu) > kBigIsland;
    int bexcl;
    const int nbig = block_scan_excl(big ? 1 : 0, bexcl, s_scan);
    const int nbw = min(nbig, min(nw - 1, (BS - nisl) / W));
    uint2* s_work = (uint2*)(lds + L.ord);
    if (tid < nisl) {
      const bool wv = big && bexcl < nbw;
      s_work[wv ? bexcl : nbw + tid - min(bexcl, nbw)] = make_uint2((uint32_t)seed, (uint32_t)off);
    }
    __syncthreads();
    const int slot = wid < nbw ? wid : nbw + tid - nbw * W;
    const uint2 job = slot < nisl ? s_work[slot] : make_uint2(0u, 0u);
    __syncthreads();
    // the walks are latency chains while other blocks' waves share the SIMDs: issue priority, as
    // for the serial walk below
    __builtin_amdgcn_s_setprio(3);
    if (wid < nbw) {
      const int sd = (int)job.x;
      int nord = (int)(job.y & 0xffffu), nb = (int)(job.y >> 16), dmax = 0;
      MACM_WALK(par_walk, sd, nord, nb, nb, dmax);
      if ((tid & (W - 1)) == 0) atomicMax(&s_misc[1], dmax);
    } else if (slot < nisl) {
      // the serial walk of island `slot` from its seed; its bodies, contacts and stack live in its
      // own ranges
      const int seed = (int)job.x;
      int nord = (int)(job.y & 0xffffu), nb = (int)(job.y >> 16), dmax = 0;
      MACM_WALK(serial_walk, seed, nord, nb, dmax);
      atomicMax(&s_misc[1], dmax);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  // The DFS is one latency chain on one wave while the block's other waves wait at the barrier
  // and other blocks' waves share the SIMD: raise its issue priority for the walk (as the wave
  // kernel does for its chain).
  if (tid < W) __builtin_amdgcn_s_setprio(3);
  if (!par_dfs && !isl_dfs && tid == 0) {  // -DMACM_NO_ISLAND_DFS: one thread walks every island
    int nord = 0, nisl = 0, nb = 0, dmax = 0;
    for (int w = (N + 63) / 64 - 1; w >= 0;) {
      const unsigned long long m = s_todo[w];  // bodies with edges not considered as seeds yet
      if (m == 0ull) {
        --w;
        continue;
      }
      const int s = w * 64 + 63 - __clzll(m);
      s_todo[w] = m & ~(1ull << (s & 63));
      if (s_last[s] & kPopped) continue;  // walked with an earlier seed's island
      s_ic[nisl] = (uint16_t)nord;
      s_ib[nisl] = (uint16_t)nb;
      MACM_WALK(serial_walk, s, nord, nb, dmax);
      ++nisl;
    }
    s_ic[nisl] = (uint16_t)nord;
    s_ib[nisl] = (uint16_t)nb;
    s_misc[0] = nisl;
    s_misc[1] = dmax;
  }
  if (par_dfs && tid < W) {  // -DMACM_NO_DFS_KERNEL: dense envs walked here by wave 0
    int nord = 0, nisl = 0, nb = 0, dmax = 0;
    for (int w = (N + 63) / 64 - 1; w >= 0;) {
      const unsigned long long m = s_todo[w] & __ballot(!(s_last[min(w * 64 + tid, N - 1)] & kPopped));
      if (m == 0ull) {
        --w;
        continue;
      }
      const int sd = w * 64 + 63 - __clzll(m);
      __builtin_amdgcn_wave_barrier();
      if (tid == 0) {
        s_ic[nisl] = (uint16_t)nord;
        s_ib[nisl] = (uint16_t)nb;
      }
      MACM_WALK(par_walk, sd, nord, nb, 0, dmax);
      ++nisl;
    }
    if (tid == 0) {
      s_ic[nisl] = (uint16_t)nord;
      s_ib[nisl] = (uint16_t)nb;
      s_misc[0] = nisl;
      s_misc[1] = dmax;
    }
  }
#undef MACM_WALK
  if (tid < W) __builtin_amdgcn_s_setprio(0);
  __syncthreads();
  const int nisl = s_misc[0];
  WSTAMP(20);
  const int nord = nisl > 0 ? (int)s_ic[nisl] : 0;

  // ---- Gauss-Seidel levels (computed by the DFS): level-order positions ----------------------
  // Contacts of one level share no body, so kernel B solves a level's contacts at once and every
  // body still sees Box2D's sequence of updates (b2ContactSolver walks the island in DFS order).
  uint32_t* s_lst = (uint32_t*)(lds + L.adj);  // [levels + 1] counts, then starts (edges are dead)
  const int nlvl = s_misc[1];
  for (int q = tid; q <= nlvl; q += BS) s_lst[q] = 0u;
  __syncthreads();
  constexpr int kPer = 5;  // tcap <= 5 * blockDim: at most 5 contacts per thread
  int slot[kPer];
#pragma unroll
  for (int m = 0; m < kPer; ++m) {
    const int k = tid + m * BS;
    slot[m] = k < nord ? (int)atomicAdd(&s_lst[s_lvl[k]], 1u) : 0;
  }
  __syncthreads();
  {  // exclusive scan of the level counts in place; thread t owns levels [t*per, (t+1)*per)
    const int per = (nlvl + BS - 1) / BS;
    const int l0 = tid * per, l1 = min(nlvl, l0 + per);
    int sum = 0;
    for (int l = l0; l < l1; ++l) sum += (int)s_lst[l];
    int run;
    block_scan_excl(sum, run, s_scan);
    for (int l = l0; l < l1; ++l) {
      const int c = (int)s_lst[l];
      s_lst[l] = (uint32_t)run;
      run += c;
    }
    if (tid == 0) s_lst[nlvl] = (uint32_t)nord;
  }
  __syncthreads();
  WSTAMP(21);

  // ---- integrate velocities; level-ordered contact records with normals -> HBM ------------
  const int IS = wg_isl_stride(N);
  if (act) {
    const float vx = v.x + P.dt * (0.0f + P.inv_mass * Fx);
    const float vy = v.y + P.dt * (0.0f + P.inv_mass * Fy);
    B.x_vmid[ag] = make_float2(vx * P.damp, vy * P.damp);
    B.x_deg[ag] = deg > 0 ? 1 : 0;
    B.x_ibod[ag] = s_ibod[tid];
  }
  float4* xc = B.x_cst + (size_t)e * tcap;
  float2* xi = B.x_cimp + (size_t)e * tcap;
  uint16_t* xo = B.x_ord + (size_t)e * tcap;
#pragma unroll
  for (int m = 0; m < kPer; ++m) {
    const int k = tid + m * BS;
    if (k >= nord) continue;
    const int t = s_ord[k];
    const uint32_t ab = s_tab[t] & 0x7fffffffu;
    const int a = ab & 0xffffu, b = ab >> 16;
    const float2 pa = s_c[a], pb = s_c[b];
    float nx = 1.0f, ny = 0.0f;
    const float ddx = pa.x - pb.x, ddy = pa.y - pb.y;
    if (ddx * ddx + ddy * ddy > kEps * kEps) {
      nx = pb.x - pa.x;
      ny = pb.y - pa.y;
      normalize(nx, ny);
    }
    // the island of contact k (kernel B's per-island position-pass exit): binary search of the
    // island contact ranges
    int lo = 0, hi = nisl - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int)s_ic[mid] <= k) lo = mid; else hi = mid - 1;
    }
    const int lv = s_lvl[k];
    const int pos = (int)s_lst[lv] + slot[m];
    xc[pos] = make_float4(__uint_as_float(ab), nx, ny, __int_as_float((lv << 16) | lo));
    xi[pos] = g_lam[t];
    xo[pos] = (uint16_t)t;
  }
  if (tid == 0) B.x_nlvl[e] = nlvl;
  WSTAMP(22);
  for (int q = tid; q <= nisl; q += BS) {
    B.x_ic[(size_t)e * IS + q] = s_ic[q];
    B.x_ib[(size_t)e * IS + q] = s_ib[q];
  }
  if (tid == 0) B.x_nisl[e] = nisl;
}

namespace wg {
// flock_dfs_wg's LDS (one wave per env): CSR edges (other body only), offsets, per-body level and
// walk state, the stack (one dummy slot past the end), the bodies with touching edges, the island
// contact starts. The level counts of the records' counting sort reuse the edges.
struct WgLayoutD {
  int adj, off, last, stk, has, ic, total;
};
__host__ __device__ inline WgLayoutD wg_layout_d(int N, int tcap) {
  WgLayoutD L;
  int o = 0;
  auto take = [&](int bytes) {
    int r = o;
    o = align16(o + bytes);
    return r;
  };
  // 2 tcap edges, the other body (10 bits, N <= 1024) three to a word; adj..stk are reused as the
  // level counts (u32 [T + 1], T <= tcap)
  const int rest = align16(2 * (N + 1)) + align16(2 * N) + align16(2 * (N + 1));
  const int packed = 4 * ((2 * tcap + 2) / 3);
  L.adj = take(packed > 4 * (tcap + 1) - rest ? packed : 4 * (tcap + 1) - rest);
  L.off = take(2 * (N + 1));
  L.last = take(2 * N);
  L.stk = take(2 * (N + 1));
  L.has = take(8 * ((N + 63) / 64));
  L.ic = take(2 * (N / 2 + 2));
  L.total = o;
  return L;
}
}  // namespace wg

// Kernel A2 (dense envs): the island DFS in Box2D order by one wave (the wave-parallel walk of
// kernel A: a popped body's edges one per lane, levels by a prefix maximum), then the Gauss-Seidel
// levels' counting sort and the level-ordered records for kernel B. Same order, levels and records
// as kernel A's walk. An edge in LDS is only its other body, 10 bits, three to a word (19.3 KB of
// LDS at C5: 8 envs per CU, all 2048 of a C5 shard resident; 4-B edges and a visited bit per
// contact took 45 KB, 3 per CU): a contact is new iff its other body has not been popped yet (the
// first of its two bodies to be popped walks it), and the walk writes the edge's CSR slot, which
// the record pass turns into the contact through x_adj.
__device__ __forceinline__ void dfs_env(const StepParams& P, const WorldBuffers& B, int tcap, int e, unsigned char* lds) {
  using namespace wg;
  const int lane = threadIdx.x, N = P.n_agents;
  const int tid = lane;  // WSTAMP
  (void)tid;
  if (B.x_nisl[e] != kDfsPending) return;  // kernel A walked it, or the spill step stepped it
  WSTAMP(26);
  const WgLayoutD L = wg_layout_d(N, tcap);
  uint32_t* s_adj = (uint32_t*)(lds + L.adj);
  uint16_t* s_off = (uint16_t*)(lds + L.off);
  uint16_t* s_last = (uint16_t*)(lds + L.last);
  uint16_t* s_stk = (uint16_t*)(lds + L.stk);
  unsigned long long* s_has = (unsigned long long*)(lds + L.has);  // bodies with touching edges
  uint16_t* s_ic = (uint16_t*)(lds + L.ic);
  const int IS = wg_isl_stride(N);
  const uint16_t* xoff = B.x_off + (size_t)e * (N + 1);
  const uint32_t* xadj = B.x_adj + (size_t)e * 2 * tcap;
  uint32_t* xdfs = B.x_dfs + (size_t)e * tcap;
  uint16_t* xibod = B.x_ibod + (size_t)e * N;
  uint16_t* xib = B.x_ib + (size_t)e * IS;
  const int T2 = xoff[N];
  for (int b = lane; b <= N; b += W) s_off[b] = xoff[b];
  for (int wq = lane; 3 * wq < T2; wq += W) {
    const int q = 3 * wq;
    const uint32_t o0 = xadj[q] >> 16, o1 = q + 1 < T2 ? xadj[q + 1] >> 16 : 0u, o2 = q + 2 < T2 ? xadj[q + 2] >> 16 : 0u;
    s_adj[wq] = o0 | (o1 << 10) | (o2 << 20);
  }
  for (int b = lane; b < N; b += W) s_last[b] = 0;
  __syncthreads();
  for (int w = 0; w < (N + 63) / 64; ++w) {
    const int b = w * 64 + lane;
    const unsigned long long m = __ballot(b < N && s_off[b + 1] > s_off[b]);
    if (lane == 0) s_has[w] = m;
  }
  __syncthreads();
  __builtin_amdgcn_s_setprio(3);
  // s_last[b]: 1 + the level of the last walked contact touching b (bits 0..13; levels <= tcap <
  // 2^14), b pushed (bit 15), b popped (bit 14). One LDS read of the other body's word gives the
  // three things an edge needs: the contact was walked iff its other body was popped (the first of
  // its two bodies to be popped walks it), the body is pushed iff it was not pushed yet, and the
  // level chain's input. A new contact's other body is pushed after it either way, so the walk
  // writes its word as level | pushed; a pop ends by writing level | pushed | popped. Seeds are the
  // highest bodies with edges not yet popped (every pushed body of an island is popped in it).
  constexpr int kPushed = 0x8000, kPopped = 0x4000, kLvl = 0x3fff;
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int nord = 0, nisl = 0, nb = 0, dmax = 0;
  for (int w = (N + 63) / 64 - 1; w >= 0;) {
    const int bw = w * 64 + lane;
    const unsigned long long m = s_has[w] & __ballot(bw < N && !(s_last[min(bw, N - 1)] & kPopped));
    if (m == 0ull) {
      --w;
      continue;
    }
    const int sd = w * 64 + 63 - __clzll(m);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      s_ic[nisl] = (uint16_t)nord;
      st_wt(xib + nisl, (uint16_t)nb);  // kernel C reads it (stored write-through)
    }
    // the body to pop next with its CSR range and level: the seed (never touched yet: level 0), then
    // the last push of the previous pop (in registers; its stack slot is dropped), else the stack's
    // top (two dependent LDS round trips)
    int sp = 1;
    int top_b = sd, top_e0 = s_off[sd], top_e1 = s_off[sd + 1], top_last = 0;
    for (;;) {
      if (top_b < 0 && sp == 0) break;
      --sp;
      int bdy, e0, e1, xcur;
      if (top_b >= 0) {
        bdy = top_b;
        e0 = top_e0;
        e1 = top_e1;
        xcur = top_last;
      } else {
        bdy = s_stk[sp];
        e0 = s_off[bdy];
        e1 = s_off[bdy + 1];
        xcur = s_last[bdy] & kLvl;
      }
      top_b = -1;
      if (lane == 0) st_wt(xibod + nb, (uint16_t)bdy);
      ++nb;
      // levels of the new contacts c_1..c_m of bdy in order: X_i = i + max(X_0, max_{j<=i}(y_j - j + 1))
      // (see par_walk in kernel A). Branch-free up to the stores: lanes past the body's last edge
      // read its last edge and take no part.
      for (int q0 = e0; q0 < e1; q0 += W) {
        const int q = min(q0 + lane, e1 - 1);
        const uint32_t qw = (uint32_t)q / 3u;
        const int o = (s_adj[qw] >> (10u * ((uint32_t)q - 3u * qw))) & 1023u;
        const int so = s_last[o];
        const int oe0 = s_off[o], oe1 = s_off[o + 1];
        const bool newc = q0 + lane < e1 && !(so & kPopped);
        const bool push = newc && !(so & kPushed);
        const unsigned long long mc = __ballot(newc), mp = __ballot(push);
        const int rank = __popcll(mc & lt) + 1;
        int z = wave_prefix_max(newc ? (so & kLvl) - rank + 1 : -0x3fffffff);
        const int xi = rank + max(xcur, z);
        if (newc) {
          s_last[o] = (uint16_t)(xi | kPushed);
          xdfs[nord + rank - 1] = (uint32_t)q | ((uint32_t)(xi - 1) << 16);  // CSR slot: < 2 tcap <= 9216
          s_stk[push ? sp + __popcll(mp & lt) : N] = (uint16_t)o;  // slot N: the dummy
        }
        const int mnew = __popcll(mc);
        if (mnew) xcur = mnew + max(xcur, __builtin_amdgcn_readlane(z, W - 1));
        nord += mnew;
        sp += __popcll(mp);
        if (mp) {  // the new top: the highest pushing lane, popped next straight from registers
          const int hl = 63 - __clzll(mp);
          top_b = __builtin_amdgcn_readlane(o, hl);
          top_e0 = __builtin_amdgcn_readlane(oe0, hl);
          top_e1 = __builtin_amdgcn_readlane(oe1, hl);
          top_last = __builtin_amdgcn_readlane(xi, hl);
        }
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) s_last[bdy] = (uint16_t)(xcur | kPushed | kPopped);
      dmax = max(dmax, xcur);
      __builtin_amdgcn_wave_barrier();
    }
    ++nisl;
  }
  if (lane == 0) {
    s_ic[nisl] = (uint16_t)nord;
    st_wt(xib + nisl, (uint16_t)nb);
  }
  __builtin_amdgcn_s_setprio(0);
  // this wave's x_dfs stores are read back below (workgroup scope: this CU, this XCD's L2)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __syncthreads();
  WSTAMP(27);

  // ---- Gauss-Seidel levels: counting sort into level order; the records for kernel B ------------
  uint32_t* s_cnt = s_adj;  // [dmax + 1] over adj..stk (dead after the walk; dmax <= T <= tcap)
  // Both passes over the walk's contacts take kDfsBatch of them per lane at a time, every global
  // load of the batch issued before the first is used: a contact's record is a chain of dependent
  // L2 reads (x_dfs -> x_adj -> x_tab -> pos), which one contact at a time left exposed
  // (round 3: 0.53 M cycles per C5 env for the sort and the records)
  constexpr int U = kDfsBatch;
  for (int l = lane; l <= dmax; l += W) s_cnt[l] = 0u;
  __syncthreads();
  for (int k0 = 0; k0 < nord; k0 += U * W) {
    uint32_t dl[U];
#pragma unroll
    for (int j = 0; j < U; ++j) dl[j] = xdfs[min(k0 + j * W + lane, nord - 1)];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (k0 + j * W + lane < nord) atomicAdd(&s_cnt[dl[j] >> 16], 1u);
  }
  __syncthreads();
  {  // exclusive scan over the levels: lane L owns levels [L per, (L + 1) per)
    const int per = (dmax + W - 1) / W;
    const int l0 = lane * per, l1 = min(dmax, l0 + per);
    int sum = 0;
    for (int l = l0; l < l1; ++l) sum += (int)s_cnt[l];
    const int incl = wave_prefix_sum(sum);
    int run = incl - sum;
    for (int l = l0; l < l1; ++l) {
      const int c = (int)s_cnt[l];
      s_cnt[l] = (uint32_t)run;
      run += c;
    }
  }
  __syncthreads();
  const uint32_t* xt = B.x_tab + (size_t)e * tcap;
  const float2* g_lam = B.scratch + (size_t)e * tcap;
  float4* xc = B.x_cst + (size_t)e * tcap;
  float2* xi = B.x_cimp + (size_t)e * tcap;
  uint16_t* xo = B.x_ord + (size_t)e * tcap;
  const float2* pos = B.pos + (size_t)e * N;
  for (int k0 = 0; k0 < nord; k0 += U * W) {
    uint32_t dl[U], abl[U];
    int tl[U];
    float2 pal[U], pbl[U], laml[U];
#pragma unroll
    for (int j = 0; j < U; ++j) dl[j] = xdfs[min(k0 + j * W + lane, nord - 1)];
#pragma unroll
    for (int j = 0; j < U; ++j) tl[j] = xadj[dl[j] & 0xffffu] & 0xffffu;  // CSR slot -> contact
#pragma unroll
    for (int j = 0; j < U; ++j) {
      abl[j] = xt[tl[j]];
      laml[j] = g_lam[tl[j]];
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      pal[j] = pos[abl[j] & 0xffffu];  // the start-of-step positions (kernel C writes them back)
      pbl[j] = pos[abl[j] >> 16];
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int k = k0 + j * W + lane;
      if (k >= nord) break;
      const uint32_t ab = abl[j];
      const int lv = dl[j] >> 16;
      const float2 pa = pal[j], pb = pbl[j];
      float nx = 1.0f, ny = 0.0f;  // InitializeVelocityConstraints: (1, 0) when the centres coincide
      const float ddx = pa.x - pb.x, ddy = pa.y - pb.y;
      if (ddx * ddx + ddy * ddy > kEps * kEps) {
        nx = pb.x - pa.x;
        ny = pb.y - pa.y;
        normalize(nx, ny);
      }
      int lo = 0, hi = nisl - 1;  // the island of contact k
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int)s_ic[mid] <= k) lo = mid; else hi = mid - 1;
      }
      const int p = (int)atomicAdd(&s_cnt[lv], 1u);  // any slot of its level: a level's contacts share no body
      xc[p] = make_float4(__uint_as_float(ab), nx, ny, __int_as_float((lv << 16) | lo));
      xi[p] = laml[j];
      xo[p] = (uint16_t)tl[j];
    }
  }
  for (int q = lane; q <= nisl; q += W) B.x_ic[(size_t)e * IS + q] = s_ic[q];
  if (lane == 0) {
    B.x_nlvl[e] = dmax;
    st_wt(B.x_nisl + e, nisl);
  }
  WSTAMP(28);
}

__global__ __launch_bounds__(64) void flock_dfs_wg(StepParams P, WorldBuffers B, int tcap) {
  extern __shared__ __align__(16) unsigned char lds[];
  dfs_env(P, B, tcap, wg_env(B), lds);
}

namespace wg {

// One Gauss-Seidel velocity constraint (b2ContactSolver::SolveVelocityConstraints, one point,
// fixedRotation bodies): the fused kernel's arithmetic.
// Kernel B's contact updates on packed (x, y) pairs (v_pk_mul_f32 / v_pk_add_f32, each lane of a pair
// the scalar form's IEEE operation, no contraction: bit-identical). Round 5: C5 -1.2%, C3 even
// (profiles/r05/abtests/wg_packed).
typedef float pf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void gs_velocity(float2& va, float2& vb, float nx, float ny, float& ln, float& ltg,
                                            float mA, float mB, float kmass, float friction) {
  pf2 vA = {va.x, va.y}, vB = {vb.x, vb.y};
  const pf2 n = {nx, ny}, t = {ny, -nx};
  {
    const pf2 pr = (vB - vA) * t;
    const float vt = pr.x + pr.y;
    float lambda = kmass * (-vt);
    const float maxf = friction * ln;
    const float ni = sclamp(ltg + lambda, -maxf, maxf);
    lambda = ni - ltg;
    ltg = ni;
    const pf2 Pv = lambda * t;
    vA = vA - mA * Pv;
    vB = vB + mB * Pv;
  }
  {
    const pf2 pr = (vB - vA) * n;
    const float vn = pr.x + pr.y;
    float lambda = -kmass * (vn - 0.0f);
    const float ni = smax(ln + lambda, 0.0f);
    lambda = ni - ln;
    ln = ni;
    const pf2 Pv = lambda * n;
    vA = vA - mA * Pv;
    vB = vB + mB * Pv;
  }
  va = make_float2(vA.x, vA.y);
  vb = make_float2(vB.x, vB.y);
}

__device__ __forceinline__ void gs_warm(float2& va, float2& vb, float nx, float ny, float ln, float lt, float mA,
                                        float mB) {
  const pf2 n = {nx, ny}, t = {ny, -nx};
  const pf2 Pv = ln * n + lt * t;
  pf2 vA = {va.x, va.y}, vB = {vb.x, vb.y};
  vA = vA - mA * Pv;
  vB = vB + mB * Pv;
  va = make_float2(vA.x, vA.y);
  vb = make_float2(vB.x, vB.y);
}

// b2PositionSolverManifold + one position-constraint correction; returns the separation.
// KPOS: K = mA + mB is known to be > 0 (else the impulse is 0, b2ContactSolver's K > 0 test).
template <bool KPOS = false>
__device__ __forceinline__ float gs_position(float2& ca, float2& cb, float radius, float mA, float mB) {
  const pf2 cA = {ca.x, ca.y}, cB = {cb.x, cb.y};
  const pf2 d = cB - cA;
  const pf2 d2 = d * d;
  const float len = sqrt_rn(d2.x + d2.y);
  const pf2 n = len < kEps ? d : d * rcp_rn(len);
  const pf2 pr = d * n;
  const float sep = (pr.x + pr.y) - radius - radius;
  const float Cc = sclamp(kBaumgarte * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
  const float K = mA + mB;
  const float imp = KPOS ? div_by_invariant(-Cc, K) : K > 0.0f ? div_by_invariant(-Cc, K) : 0.0f;
  const pf2 Pv = imp * n;
  const pf2 nA = cA - mA * Pv, nB = cB + mB * Pv;
  ca = make_float2(nA.x, nA.y);
  cb = make_float2(nB.x, nB.y);
  return sep;
}

}  // namespace wg

// Kernel B: one wave per env solves all its islands together, level by level (kernel A's
// Gauss-Seidel levels): a level's contacts touch disjoint bodies, so lanes solve them at once
// and each body gets Box2D's sequence of updates (b2Island::Solve -> b2ContactSolver). The
// passes are Box2D's: warm start, vel_iters velocity passes, StoreImpulses, position
// integration, up to pos_iters position passes with each island leaving after the first pass
// whose minimum separation is >= -3 linearSlop.
//
// A level step is one straight block: every lane runs it, the lanes outside the level on a dummy
// LDS slot of their own (no exec-mask branch), the next level's addresses selected while this
// level solves. Level steps are issue- and latency-bound (one wave per SIMD pair at C5:
// tools/ubench_level.hip), so the loops run two levels per iteration (no register rotation or
// back-edge per level) and the position passes keep no uniform K > 0 branch inside the loop.
__device__ __forceinline__ void solve_env(const StepParams& P, const WorldBuffers& B, int tcap, int e,
                                          unsigned char* lds) {
  using namespace wg;
  const int lane = threadIdx.x, N = P.n_agents;
  const int IS = wg_isl_stride(N);
  float2* s_v = (float2*)lds;
  float2* s_c = s_v + N;
  float* s_mins = (float*)(s_c + N);          // [IS] per island: minimum separation of the pass
  uint8_t* s_done = (uint8_t*)s_mins + wg_solve_mins_bytes(N);  // [IS] per island: position-solved
  float2* s_dum = (float2*)s_mins;  // [W] the velocity passes' dummy slots (s_mins is set per position pass)
  const size_t en = (size_t)e * N;
  const int nisl = B.x_nisl[e];
  if (nisl < 0) return;  // stepped whole by the spill step in kernel A
  const int nc = nisl > 0 ? (int)B.x_ic[(size_t)e * IS + nisl] : 0;
  const int nch = (nc + W - 1) / W;
  const float4* cst = B.x_cst + (size_t)e * tcap;
  float2* cimp = B.x_cimp + (size_t)e * tcap;
  const uint16_t* xord = B.x_ord + (size_t)e * tcap;
  float2* g_lam = B.scratch + (size_t)e * tcap;
  for (int i = lane; i < N; i += W) {
    s_c[i] = B.pos[en + i];
    s_v[i] = B.x_vmid[en + i];
  }
  for (int I = lane; I < nisl; I += W) s_done[I] = 0;
  __syncthreads();
  const int tid = lane;  // for WSTAMP (slots 13..15, diagnostic build)
  (void)tid;
  WSTAMP(13);
  const float mA = P.inv_mass, mB = P.inv_mass;
  const float kmass = (mA + mB) > 0.0f ? 1.0f / (mA + mB) : 0.0f;
  const float friction = P.friction;

  // The records are in level order (record.w = level << 16 | island). The wave walks them in
  // chunks of 64, one record per lane, loaded a chunk ahead; inside a chunk it steps through the
  // chunk's levels, the lanes of the current level solving together. A level that continues into
  // the next chunk is finished there (its contacts share no body, so the split is harmless).
  // Between level steps the next lanes must see this step's body updates (wave_lds_sync: a wave's
  // LDS accesses are performed in issue order).
  auto level_sync = [&]() { wave_lds_sync(); };
  // Chunk loads are branch-free (lanes past the end re-read the last record) and waited for
  // explicitly at the end of the chunk before: the compiler then places no memory wait inside the
  // level loop.
  auto wait_vm = [&]() { __builtin_amdgcn_s_waitcnt(0x0f70); };  // vmcnt(0)
  struct Slot {
    float4 r;
    float2 m;
    int o;
  };
  auto load = [&](int c, Slot& x) {
    const int k = min(c * W + lane, nc - 1);
    x.r = cst[k];
    x.m = cimp[k];
    x.o = xord[k];
  };
  // a lane's level (past the end: a level no chunk walks) and the chunk's first / last level
  auto chunk_levels = [&](int c, const Slot& x, int& mylv, int& lv0, int& lv1) {
    mylv = c * W + lane < nc ? __float_as_int(x.r.w) >> 16 : 0x7fff;
    const int last = min(W, nc - c * W) - 1;
    lv0 = __builtin_amdgcn_readfirstlane(mylv);
    lv1 = __builtin_amdgcn_readlane(mylv, last);
  };
  // Steps levels lv0..lv1 of a chunk: step(lv, on) with the addresses it reads / writes chosen one
  // step ahead by addr(on) (on: this lane's record is at that level); two steps per iteration
  auto level_loop = [&](int lv0, int lv1, int mylv, auto&& step) {
    bool on = mylv == lv0;
    int lv = lv0;
    for (; lv < lv1; lv += 2) {
      step(lv, on, mylv == lv + 1);
      level_sync();
      step(lv + 1, mylv == lv + 1, mylv == lv + 2);
      level_sync();
      on = mylv == lv + 2;
    }
    if (lv == lv1) {
      step(lv, on, false);
      level_sync();
    }
  };

  // Warm start and velocity passes. last: the final impulses go straight to list order (g_lam).
  // warm is a compile-time flag (BoolC-like): no branch inside a level step
  auto vel_pass = [&](auto warm_c, bool last) {
    constexpr bool warm = decltype(warm_c)::value;
    if (nch == 0) return;
    Slot cur, nxt;
    load(0, cur);
    wait_vm();
    for (int c = 0; c < nch; ++c) {
      load(c + 1, nxt);
      int mylv, lv0, lv1;
      chunk_levels(c, cur, mylv, lv0, lv1);
      const uint32_t ab = __float_as_uint(cur.r.x);
      const int a = ab & 0xffffu, b = ab >> 16;
      float2 im = cur.m;
      // every lane runs every level step, the lanes outside the level on their own dummy slot (no
      // exec-mask branch per level); only the level's lanes keep their impulses
      float2* const pa0 = s_v + a;
      float2* const pb0 = s_v + b;
      float2* const pd = s_dum + 0;  // shared: an LDS broadcast for the idle lanes
      float2* pa = mylv == lv0 ? pa0 : pd;
      float2* pb = mylv == lv0 ? pb0 : pd;
      level_loop(lv0, lv1, mylv, [&](int, bool onc, bool onn) {
        float2 va = *pa, vb = *pb;
        // the next level's addresses are selected while this level solves (off the read's path)
        float2* const na = onn ? pa0 : pd;
        float2* const nb = onn ? pb0 : pd;
        float lx = im.x, ly = im.y;
        if constexpr (warm) gs_warm(va, vb, cur.r.y, cur.r.z, lx, ly, mA, mB);
        else gs_velocity(va, vb, cur.r.y, cur.r.z, lx, ly, mA, mB, kmass, friction);
        *pa = va;
        *pb = vb;
        im.x = onc ? lx : im.x;
        im.y = onc ? ly : im.y;
        pa = na;
        pb = nb;
      });
      const int k = c * W + lane;
      if (!warm && k < nc) {
        if (last) st_wt(g_lam + cur.o, im);  // kernel C reads it (the handoff)
        else cimp[k] = im;
      }
      wait_vm();
      cur = nxt;
    }
  };
  if (P.warm_starting) vel_pass(std::true_type{}, false);
  for (int it = 0; it < P.vel_iters; ++it) vel_pass(std::false_type{}, it + 1 == P.vel_iters);
  if (P.vel_iters == 0)  // StoreImpulses of the (warm-started) impulses as they are
    for (int k = lane; k < nc; k += W) st_wt(g_lam + xord[k], cimp[k]);

  WSTAMP(14);
  // ---- integrate positions ---------------------------------------------------------------------
  for (int i = lane; i < N; i += W) {
    const float2 vv = s_v[i];
    float vx = vv.x, vy = vv.y;
    const float tx = P.dt * vx, ty = P.dt * vy;
    if (tx * tx + ty * ty > kMaxTranslation * kMaxTranslation) {
      const float ratio = kMaxTranslation / sqrtf(tx * tx + ty * ty);
      vx = vx * ratio;
      vy = vy * ratio;
    }
    const float2 c = s_c[i];
    s_c[i] = make_float2(c.x + P.dt * vx, c.y + P.dt * vy);
    st_wt(B.x_vout + en + i, make_float2(vx, vy));
  }
  __syncthreads();

  // ---- position passes: every island not yet solved, level by level; an island is solved after
  //      the first pass whose minimum separation (starting at 0) is >= -3 linearSlop. The minimum
  //      is an LDS float min (ds_min_f32): the separations are finite, a NaN one would be ignored
  //      as by the order-preserving integer keys it replaces (round 3) ----------------------------
  // K = mA + mB > 0 for every dynamic body (fill_body_params: a zero mass becomes 1); the K <= 0
  // form (b2ContactSolver's `K > 0 ? -C / K : 0`) exists for an infinite density only and keeps
  // the test out of the level step.
  auto pos_passes = [&](auto kpos_c) {
    constexpr bool kpos = decltype(kpos_c)::value;
    for (int it = 0; it < P.pos_iters; ++it) {
      for (int I = lane; I < nisl; I += W) s_mins[I] = 0.0f;
      __syncthreads();
      Slot cur, nxt;
      if (nch > 0) load(0, cur);
      wait_vm();
      for (int c = 0; c < nch; ++c) {
        load(c + 1, nxt);
        int mylv, lv0, lv1;
        chunk_levels(c, cur, mylv, lv0, lv1);
        const int I = __float_as_int(cur.r.w) & 0xffff;
        const uint32_t ab = __float_as_uint(cur.r.x);
        const int a = ab & 0xffffu, b = ab >> 16;
        const bool live = !s_done[I];
        // branch-free level steps as in the velocity passes; the dummy slots are in s_v (dead after
        // the position integration), a dummy lane's minimum goes to its slot's first word
        float2* const pdd = s_v + 0;
        // a dummy lane's minimum stays in a word of its own (atomics on one address serialise)
        float* const pmd = reinterpret_cast<float*>(s_v + 1 + lane);
        const int mylvp = live ? mylv : -1;
        float2* const pca = s_c + a;
        float2* const pcb = s_c + b;
        float* const pmi = s_mins + I;
        float2* pa = mylvp == lv0 ? pca : pdd;
        float2* pb = mylvp == lv0 ? pcb : pdd;
        float* pm = mylvp == lv0 ? pmi : pmd;
        level_loop(lv0, lv1, mylvp, [&](int, bool, bool onn) {
          float2 ca = *pa, cb = *pb;
          float2* const na = onn ? pca : pdd;
          float2* const nb = onn ? pcb : pdd;
          float* const nm = onn ? pmi : pmd;
          const float sep = gs_position<kpos>(ca, cb, P.radius, mA, mB);
          *pa = ca;
          *pb = cb;
          __hip_atomic_fetch_min(pm, sep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
          pa = na;
          pb = nb;
          pm = nm;
        });
        wait_vm();
        cur = nxt;
      }
      __syncthreads();
      bool open = false;
      for (int I = lane; I < nisl; I += W) {
        if (s_done[I]) continue;
        if (s_mins[I] >= -3.0f * kLinearSlop) s_done[I] = 1;
        else open = true;
      }
      const bool any_open = __ballot(open) != 0ull;
      __syncthreads();
      if (!any_open) break;
    }
  };
  if (mA + mB > 0.0f) pos_passes(std::true_type{});
  else pos_passes(std::false_type{});
  uint8_t* isolv = B.x_isolv + (size_t)e * IS;
  for (int I = lane; I < nisl; I += W) st_wt(isolv + I, s_done[I]);
  WSTAMP(15);
#ifdef MACM_STAMPS
  if (lane == 0) B.stamps[(size_t)e * 32 + 12] = (unsigned long long)B.x_nlvl[e] | ((unsigned long long)nc << 32);
#endif
  for (int i = lane; i < N; i += W) st_wt(B.x_cout + en + i, s_c[i]);
}

// Kernel B: one wave per env. Measured slower and removed in round 6 (evidence kept,
// profiles/r05/abtests/): the dense envs' DFS fused into this kernel (handoff_fused), and two envs per
// wave (solve_pair).
__global__ __launch_bounds__(64) void flock_solve_wg(StepParams P, WorldBuffers B, int tcap, Handoff H) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = wg_env(B);
  const HandoffPublish publish(H, e);  // to kernel C when this body ends (any return)
  solve_env(P, B, tcap, e, lds);
}

template <typename OT>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void flock_step_wg_c(StepParams P, WorldBuffers B, int cur, int tcap,
                                                        OT* __restrict__ obs, int32_t* __restrict__ nbr_out,
                                                        float* __restrict__ rew_out, uint8_t* __restrict__ coll_out,
                                                        uint8_t* __restrict__ done_out, Handoff H,
                                                        uint8_t* __restrict__ bot_act) {
  using namespace wg;
  extern __shared__ __align__(16) unsigned char lds[];
  // in kernel B's finish order (the block scan's scratch words carry the env to the block)
  const int e = H.q ? handoff_take(B, H, reinterpret_cast<int*>(lds + wg_layout_c(P.n_agents).scan)) : wg_env(B);
  if (e < 0) {
    // this block cannot know which env it missed: every env carries the bit, so
    // macm_world_status shows the world's results as invalid wherever they were read
    for (int i = threadIdx.x; i < P.n_envs; i += blockDim.x) atomicOr(&B.status[i], (int)MACM_ST_HANDOFF);
    return;
  }
  const int tid = threadIdx.x;
  const int BS = blockDim.x;
  const int N = P.n_agents;
  const int C = P.max_contacts;
  const bool act = tid < N;
  const size_t ag = (size_t)e * N + tid;
  const int nxt = cur ^ 1;
  const WgLayoutC L = wg_layout_c(N);
  float* s_slp = (float*)(lds + L.slp);
  uint8_t* s_flag = (uint8_t*)(lds + L.flags);
  uint32_t* s_oldc = (uint32_t*)(lds + L.oldc);
  int* s_scan = (int*)(lds + L.scan);
  int* s_misc = (int*)(lds + L.misc);
  float4* s_fn = (float4*)(lds + L.fn);
  float4* s_fo = (float4*)(lds + L.fo);
  float2* s_c = (float2*)(lds + L.c);
  uint32_t* s_pk = (uint32_t*)(lds + L.pk);
  uint16_t* s_bjv = (uint16_t*)(lds + L.bjv);
  const float2* g_lam = B.scratch + (size_t)e * tcap;
  const int IS = wg_isl_stride(N);
  // with the handoff, the island count and B's solve outputs are read write-through (flock_dfs_wg
  // stores the count so)
  const bool hwt = H.q != nullptr;
  const int nisl = hwt ? ld_wt(B.x_nisl + e) : B.x_nisl[e];
  if (nisl < 0) {  // stepped whole by the spill step in kernel A (its observation is written)
    if (bot_act && obs && act) {
      const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
      bot_flock_row<OT>(obs + ag * od, od, bot_act + ag * 3);
    }
    return;
  }
  WSTAMP(0);

  const uint32_t* cab = B.cab[cur] + (size_t)e * C;
  const int step_count = B.step_count[e];
  const int M = B.ccount[cur][e];
  float2 p = make_float2(0.0f, 0.0f);
  float slp = 0.0f, cx = 0.0f, cy = 0.0f, vx = 0.0f, vy = 0.0f;
  float4 fo = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  bool hasdeg = false;
  if (act) {
    p = B.pos[ag];
    fo = B.fat[ag];
    slp = B.sleep[ag];
    const float2 c = ld_wt(B.x_cout + ag), vv = ld_wt(B.x_vout + ag);  // kernel B's (write-through)
    cx = c.x; cy = c.y; vx = vv.x; vy = vv.y;
    hasdeg = B.x_deg[ag] != 0;
  }
  for (int q = tid; q < (N + 31) / 32; q += BS) s_oldc[q] = 0u;
  if (tid < 8) s_misc[tid] = 0;
  int status = 0;
  __syncthreads();
  for (int k = tid; k < M; k += BS) {  // agents in the old list (world.contacts before the step)
    const uint32_t ab = cab[k];
    const int a = ab & 0xffffu, b = ab >> 16;
    atomicOr(&s_oldc[a >> 5], 1u << (a & 31));
    atomicOr(&s_oldc[b >> 5], 1u << (b & 31));
  }

  // ---- sleep clock + island sleep decision --------------------------------------------------------
  float ns = 0.0f;
  if (act) {
    const bool moving = vx * vx + vy * vy > kLinearSleepTol * kLinearSleepTol;
    ns = moving ? 0.0f : slp + P.dt;
    s_slp[tid] = ns;
    s_flag[tid] = (!hasdeg && ns >= kTimeToSleep && P.pos_iters > 0) ? 1 : 0;
  }
  __syncthreads();
  WSTAMP(1);
  {
    // island sleep (b2Island::Solve's minSleepTime): one thread per island body; the island of
    // body slot k is found by binary search over the island ranges (copied to LDS), the minimum
    // by LDS atomicMin on the float bits (sleep clocks are >= 0, so their bit patterns order as
    // the floats). Scratch: the grid's entry / bucket arrays, not yet in use.
    const uint16_t* ib = B.x_ib + (size_t)e * IS;
    const uint16_t* ibod = B.x_ibod + (size_t)e * N;
    const uint8_t* isolv = B.x_isolv + (size_t)e * IS;
    uint16_t* s_ib = (uint16_t*)(lds + L.gent);     // [nisl + 1] <= N / 2 + 2 (gent: 16 N bytes)
    uint32_t* s_mn = (uint32_t*)(lds + L.gstart);   // [nisl] <= N / 2 (gstart: >= 8 N bytes)
    for (int I = tid; I <= nisl; I += BS) s_ib[I] = hwt ? ld_wt(ib + I) : ib[I];
    for (int I = tid; I < nisl; I += BS) s_mn[I] = 0x7f7fffffu;  // FLT_MAX, as the serial minimum starts
    __syncthreads();
    const int nb = nisl > 0 ? s_ib[nisl] : 0;
    for (int k = tid; k < nb; k += BS) {
      int lo = 0, hi = nisl - 1;  // the island I with ib[I] <= k < ib[I + 1]
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_ib[mid] <= k) lo = mid; else hi = mid - 1;
      }
      atomicMin(&s_mn[lo], __float_as_uint(s_slp[hwt ? ld_wt(ibod + k) : ibod[k]]));
    }
    __syncthreads();
    for (int k = tid; k < nb; k += BS) {
      int lo = 0, hi = nisl - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_ib[mid] <= k) lo = mid; else hi = mid - 1;
      }
      s_flag[hwt ? ld_wt(ibod + k) : ibod[k]] = (__uint_as_float(s_mn[lo]) >= kTimeToSleep && ld_wt(isolv + lo)) ? 1 : 0;
    }
  }
  __syncthreads();
  WSTAMP(2);

  // ---- SynchronizeFixtures ----------------------------------------------------------------------
  float4 fn = fo;
  if (act) {
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
    if (s_flag[tid]) {
      vx = 0.0f;
      vy = 0.0f;
      ns = 0.0f;
    }
    s_fn[tid] = fn;
    s_fo[tid] = fo;
    s_c[tid] = make_float2(cx, cy);
    // final velocity, sleep clock and fat AABB (nothing below reads them back; frees registers
    // for the sweep)
    B.vel[ag] = make_float2(vx, vy);
    B.fat[ag] = fn;
    B.sleep[ag] = ns;
  }
  __syncthreads();
  WSTAMP(3);

  // ---- pair sweep over the spatial hash (flock_grid.hpp): collisions, new-pair counts, nearest
  //      neighbour. Candidates of a body are the bodies of the 3 x 3 cell block around it; an env
  //      whose positions or extents the hash cannot bin takes the all-pairs sweep.
  const grid::Lds G{(float*)(lds + L.gred), (float*)(lds + L.gpar), (uint32_t*)(lds + L.gstart),
                    (float4*)(lds + L.gent), (uint32_t*)(lds + L.gsext), grid::buckets(N)};
  bool coll = act && ((s_oldc[tid >> 5] >> (tid & 31)) & 1u);
  int newcnt = 0;
  float best = __builtin_inff();
  int bj = tid == 0 ? 1 : 0;
  // strip cells from N = 256 (grid::kCellsMinAgents): with per-strip extent pruning (round 4) they
  // walk ~290 of C5's 1024 bodies per body and beat the all-pairs sweep at C3 too
  const bool cells = P.sweep == 1 || (P.sweep == 0 && N >= grid::kCellsMinAgents);
  const bool gok = cells && grid::build(G, act, make_float2(cx, cy), fn);
  WSTAMP(4);
  // Thread t sweeps the body of strip-sorted entry t (flock_grid.hpp): body i, its wave's tile of
  // strips [s0, s1], walked with broadcast reads. Results go to LDS per body (s_pk: collided bit
  // 31 | new-pair count, s_slp: best d2, s_bjv: neighbour), read back by the owning thread.
  int ti = 0, ts0 = 1, ts1 = 0;
  bool ti_over = false;  // the swept body (ti) has more new partners than np2 holds
  uint32_t np2 = 0u;     // this thread's body's last two new partners (cells path)
  if (gok) {
    const float4 E = act ? G.ent[tid] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int i = __float_as_int(E.z);
    const float px = E.x, py = E.y;
    const float4 fni = s_fn[i], foi = s_fo[i];
    grid::Tile T;
    grid::tile(G, act, px, fmaxf(fmaxf(px - fni.x, fni.z - px), 0.0f), T);
    ti = i;
    ts0 = T.s0;
    ts1 = T.s1;
    float bst = __builtin_inff();
    int bjj = i == 0 ? 1 : 0;
    bool col = false;
    int nc = 0;
    np2 = 0u;  // the last two new partners j > i, 10 bits each (most bodies have none)
#ifdef MACM_STAMPS
    int ncand = 0;
#endif
    // the walked strips in runs of consecutive strips (a run is one range of sorted entries)
    for (int b = 0; 64 * b <= T.s1 - T.s0; ++b) {
      unsigned long long m = grid::batch(G, T, b);
      while (m) {
        const int a = __ffsll((long long)m) - 1;
        const unsigned long long rest = ~(m >> a);  // the run ends at the first 0 bit from a
        const int len = rest == 0ull ? 64 - a : __ffsll((long long)rest) - 1;
        m = (a + len >= 64) ? 0ull : (m & ~((1ull << (a + len)) - 1ull));
        const int sa = T.s0 + 64 * b + a;
        const int q0 = (int)G.start[sa], q1 = (int)G.start[sa + len];
#ifdef MACM_STAMPS
        ncand += q1 - q0;
#endif
        // One candidate: its entry (position, body) and its new fat AABB. Branch-free but for the
        // rare overlap with a higher body (the old AABB's test for a new pair).
        auto cand = [&](const float4 Eq, const float4 Fj) {
          const int j = __float_as_int(Eq.z);
          const bool ovn = !(sep_max(fni, Fj) > 0.0f);
          const float dx = Eq.x - px, dy = Eq.y - py;
          const bool other = j != i;
          const float d2 = dx * dx + dy * dy;
          // grid::nn_take with bitwise operators: no short-circuit branches
          const bool take = other & ((d2 < bst) | ((d2 == bst) & (j < bjj)));
          bst = take ? d2 : bst;
          bjj = take ? j : bjj;
          col |= other & ovn;
          const bool nw = j > i && ovn && sep_max(foi, s_fo[j]) > 0.0f;
          np2 = nw ? (np2 << 10) | (uint32_t)j : np2;
          nc += nw ? 1 : 0;
        };
        // two candidates per iteration, each entry read one candidate ahead (into the register
        // pair the other candidate is not using, so the loop carries no copies that would wait
        // for the loads): an entry's read hides under the previous candidate's test
        if (q0 < q1) {
          float4 Ea = G.ent[q0];
          for (int q = q0;; q += 2) {
            const float4 Eb = G.ent[min(q + 1, q1 - 1)];
            cand(Ea, s_fn[__float_as_int(Ea.z)]);
            if (q + 1 >= q1) break;
            Ea = G.ent[min(q + 2, q1 - 1)];
            cand(Eb, s_fn[__float_as_int(Eb.z)]);
            if (q + 2 >= q1) break;
          }
        }
      }
    }
    // nearest neighbours the walked strips cannot certify (a body outside the core [c0, c1] may be
    // nearer; e.g. a body that strayed from its converged flock): the wave widens the core by 1, 2,
    // 4, ... strips each way and walks the added strips for those lanes until each is certified
    // (strips seen before change nothing); the whole range is covered after log2(H) rounds
    bool need = act && !grid::certified(G, px, T.c0, T.c1, bst);
#ifdef MACM_STAMPS
    if (need) atomicAdd(&s_misc[3], 1);
#endif
    for (int c0 = T.c0, c1 = T.c1, k = 1; __ballot(need); k <<= 1) {
      const int n0 = max(0, c0 - k), n1 = min(G.H - 1, c1 + k);
      const int qa = (int)G.start[n0], qb = (int)G.start[c0], qc = (int)G.start[c1 + 1], qd = (int)G.start[n1 + 1];
      for (int q = qa; q < qb; ++q) {
        const float4 Eq = G.ent[q];
        const int j = __float_as_int(Eq.z);
        const float dx = Eq.x - px, dy = Eq.y - py;
        if (need && j != i) grid::nn_take(j, dx * dx + dy * dy, bst, bjj);
      }
      for (int q = qc; q < qd; ++q) {
        const float4 Eq = G.ent[q];
        const int j = __float_as_int(Eq.z);
        const float dx = Eq.x - px, dy = Eq.y - py;
        if (need && j != i) grid::nn_take(j, dx * dx + dy * dy, bst, bjj);
      }
      c0 = n0;
      c1 = n1;
      need = need && !grid::certified(G, px, c0, c1, bst);
    }
#ifdef MACM_STAMPS
    if (act) atomicAdd(&s_misc[2], ncand);
#endif
    if (act) {
      s_slp[i] = bst;
      s_bjv[i] = (uint16_t)bjj;
      // collided bit 31 | new-pair count (11 bits, <= N - 1) | the last two new partners
      s_pk[i] = (col ? 0x80000000u : 0u) | ((uint32_t)nc << 20) | (np2 & 0xfffffu);
    }
    ti_over = act && nc > 2;
    __syncthreads();
    if (act) {
      const uint32_t pk = s_pk[tid];
      coll |= (pk >> 31) != 0;
      newcnt = (int)((pk >> 20) & 0x7ffu);
      np2 = pk & 0xfffffu;
      best = s_slp[tid];
      bj = s_bjv[tid];
    }
  } else if (act) {
    // The new partners j > tid come out of this ascending sweep; the first kNewSlots of them go to
    // this body's slots of an LDS scratch (the cells' entry array, unused on this path), so the
    // list build below writes them back in descending order without a second sweep.
    uint16_t* np = (uint16_t*)(lds + L.gent) + tid * kNewSlots;
#pragma unroll 2
    for (int j = 0; j < N; ++j) {
      const float4 rfn = s_fn[j];
      const float2 rc = s_c[j];
      const bool ovn = !(sep_max(fn, rfn) > 0.0f);
      const float dx = rc.x - cx, dy = rc.y - cy;
      const float d2 = dx * dx + dy * dy;
      const bool other = j != tid;
      coll |= other && ovn;
      if (other && d2 < best) {
        best = d2;
        bj = j;
      }
      if (j > tid && ovn && sep_max(fo, s_fo[j]) > 0.0f) {
        if (newcnt < kNewSlots) np[newcnt] = (uint16_t)j;
        ++newcnt;
      }
    }
  }
  // ---- next ordered list: new pairs (a desc, b desc) ++ surviving old pairs ------------------------
  WSTAMP(5);
  uint32_t* ocab = B.cab[nxt] + (size_t)e * C;
  float2* ocimp = B.cimp[nxt] + (size_t)e * C;
  int excl;
  const int nnew = block_scan_excl(newcnt, excl, s_scan);
  if (gok && nnew <= 2 * N) {
    // Bodies with one or two new partners have them in np2 (the sweep kept them). For the rare
    // body with more, its wave walks its tile again (same mapping), collecting the partners into
    // the body's segment of an LDS scratch (the dead sleep-clock array: 2N u16 slots; s_bjv holds
    // the segment starts), which the owner sorts descending. About 50 of a C5 env's 1024 bodies get
    // a new pair per step, and a body with more than two is a few per step: the walk of every wave
    // (round 3) was 28% of kernel C at C5.
    uint16_t* s_np = (uint16_t*)s_slp;
    if (act) s_bjv[tid] = (uint16_t)excl;
    __syncthreads();
    if (__ballot(ti_over)) {
      const int i = ti;
      const float4 fni = s_fn[i], foi = s_fo[i];
      const int q0 = ts0 <= ts1 ? (int)G.start[ts0] : 0, q1 = ts0 <= ts1 ? (int)G.start[ts1 + 1] : 0;
      int w = ti_over ? (int)s_bjv[i] : 0;
      for (int q = q0; q < q1; ++q) {
        const int j = __float_as_int(G.ent[q].z);
        if (ti_over && j > i && !(sep_max(fni, s_fn[j]) > 0.0f) && sep_max(foi, s_fo[j]) > 0.0f)
          s_np[w++] = (uint16_t)j;
      }
    }
    __syncthreads();
    if (act && newcnt > 0 && newcnt <= 2) {  // from np2, descending
      const uint32_t pa = np2 & 0x3ffu, pb = (np2 >> 10) & 0x3ffu;
      const uint32_t hi = newcnt == 1 ? pa : max(pa, pb), lo = min(pa, pb);
      const int w = nnew - excl - newcnt;
      if (w < C) {
        ocab[w] = (uint32_t)tid | (hi << 16);
        ocimp[w] = make_float2(0.0f, 0.0f);
      }
      if (newcnt == 2 && w + 1 < C) {
        ocab[w + 1] = (uint32_t)tid | (lo << 16);
        ocimp[w + 1] = make_float2(0.0f, 0.0f);
      }
    } else if (act && newcnt > 2) {
      uint16_t* seg = s_np + excl;
      for (int a = 1; a < newcnt; ++a) {  // insertion sort, descending
        const uint16_t x = seg[a];
        int b = a - 1;
        for (; b >= 0 && seg[b] < x; --b) seg[b + 1] = seg[b];
        seg[b + 1] = x;
      }
      int w = nnew - excl - newcnt;
      for (int t = 0; t < newcnt; ++t, ++w)
        if (w < C) {
          ocab[w] = (uint32_t)tid | ((uint32_t)seg[t] << 16);
          ocimp[w] = make_float2(0.0f, 0.0f);
        }
    }
  } else if (act && newcnt > 0 && !gok && newcnt <= kNewSlots) {  // all-pairs: from the slots, reversed
    const uint16_t* np = (const uint16_t*)(lds + L.gent) + tid * kNewSlots;
    int w = nnew - excl - newcnt;
    for (int t = newcnt - 1; t >= 0; --t, ++w)
      if (w < C) {
        ocab[w] = (uint32_t)tid | ((uint32_t)np[t] << 16);
        ocimp[w] = make_float2(0.0f, 0.0f);
      }
  } else if (act && newcnt > 0) {  // more new pairs than the scratch holds: a descending sweep
    int w = nnew - excl - newcnt;
    for (int j = N - 1; j > tid; --j) {
      if (!(sep_max(fn, s_fn[j]) > 0.0f) && sep_max(fo, s_fo[j]) > 0.0f) {
        if (w < C) {
          ocab[w] = (uint32_t)tid | ((uint32_t)j << 16);
          ocimp[w] = make_float2(0.0f, 0.0f);
        }
        ++w;
      }
    }
  }
  const float rr = (P.radius + P.radius) * (P.radius + P.radius);
  WSTAMP(6);
  int kept = 0, Tr = 0;
  for (int k0 = 0; k0 < M; k0 += BS) {
    const int k = k0 + tid;
    bool keep = false, touch = false;
    uint32_t ab = 0u;
    if (k < M) {
      ab = cab[k];
      const int a = ab & 0xffffu, b = ab >> 16;
      keep = overlap(s_fn[a], s_fn[b]);
      const float2 pa = B.pos[(size_t)e * N + a], pb = B.pos[(size_t)e * N + b];
      const float dx = pb.x - pa.x, dy = pb.y - pa.y;
      touch = !(dx * dx + dy * dy > rr);
    }
    // one block scan for both ranks (touching in the low half, kept in the high; counts <= BS)
    int packed;
    const int pn = block_scan_excl((touch ? 1 : 0) | (keep ? 0x10000 : 0), packed, s_scan);
    const int tpos = packed & 0xffff, kpos = packed >> 16, tn = pn & 0xffff, kn = pn >> 16;
    if (keep) {
      const int w = nnew + kept + kpos;
      const int trank = Tr + tpos;
      if (w < C) {
        ocab[w] = ab;
        ocimp[w] = (touch && trank < tcap) ? ld_wt(g_lam + trank) : make_float2(0.0f, 0.0f);
      }
    }
    Tr += tn;
    kept += kn;
  }
  int total = nnew + kept;
  if (total > C) {
    status |= MACM_ST_CONTACT_OVERFLOW;
    total = C;
  }

  // ---- rewards + obs -----------------------------------------------------------------------------
  WSTAMP(7);
  float rew = 0.0f;
  if (act) {
    const float2 tg = B.targets[(size_t)e * P.n_targets + B.tidx[tid]];
    const float ang = B.angle[ag];
    const float tdx = tg.x - cx, tdy = tg.y - cy;
    const float td2 = tdx * tdx + tdy * tdy;
    const double d = sqrt((double)td2);
    if (coll) rew = -1.0f;
    else if (P.reward_mode == MACM_REWARD_LINEAR) rew = (float)((-d / 35) + 1);
    else rew = (d < P.reward_radius) ? 1.0f : 0.0f;
    rew_out[ag] = rew;
    if (coll_out) coll_out[ag] = coll ? 1 : 0;
    if (nbr_out) nbr_out[ag] = bj;
    if (obs) {
      const int od = P.coord == MACM_COORD_CARTESIAN ? 6 : 4;
      const float2 cb = s_c[bj];
      write_obs<OT>(obs + ag * od, P.coord, ang, best, cb.x - cx, cb.y - cy, tdx, tdy, td2);
      // the closed loop's next action (bots.flock on the row as stored: this thread's own stores)
      if (bot_act) bot_flock_row<OT>(obs + ag * od, od, bot_act + ag * 3);
    }
  }
  int dummy;  // both counts in one scan (collided in the low half, rewarded in the high)
  const int cp = block_scan_excl((act && coll ? 1 : 0) | (act && rew > 0.0f ? 0x10000 : 0), dummy, s_scan);
  const int ncoll = cp & 0xffff, npos = cp >> 16;
  const bool lin = P.reward_mode == MACM_REWARD_LINEAR;  // binary steps: c2 - c1 (macm_world_reward_sums)
  const double rsum = lin ? block_pairwise_sum((double)rew, reinterpret_cast<double*>(s_scan)) : 0.0;  // thread 0
  if (status) atomicOr(&s_misc[1], status);
  __syncthreads();
  WSTAMP(8);
  if (act) {
    B.pos[ag] = make_float2(cx, cy);
  }
  if (tid == 0) {
    const int nst = s_misc[1];
    const double tp = B.time_passed[e] + P.inv_hz;
    const uint8_t dn = tp > P.time_limit ? 1 : 0;
    B.time_passed[e] = tp;
    B.done[e] = dn;
    if (done_out) done_out[e] = dn;
    B.step_count[e] = step_count + 1;
    B.ccount[nxt][e] = total;
    if (nst) {
      B.status[e] |= nst;
      report_status(B, nst);
    }
    unsigned long long* ec = B.env_counters + (size_t)e * 4;
    ec[0] += (unsigned long long)N;
    ec[1] += (unsigned long long)ncoll;
    ec[2] += (unsigned long long)npos;
    ec[3] += (unsigned long long)dn;
    if (lin) add_reward_sum(B, e, rsum);
  }
  WSTAMP(9);
#ifdef MACM_STAMPS
  if (tid == 0) {  // strip diagnostics: tile candidates per body (x1000), bodies walking all strips
    B.stamps[(size_t)e * 32 + 10] = (unsigned long long)s_misc[2] * 1000ull / N;
    B.stamps[(size_t)e * 32 + 11] = (unsigned long long)s_misc[3];
  }
#endif
}

// ---- launchers -------------------------------------------------------------------------------------
int wg_block(int N) { return ((N + 63) / 64) * 64; }
int wg_init_lds_bytes(int N) { return align16((int)sizeof(wg::Rec) * N) + 4 * 32; }
// kernel A's dynamic LDS: its own layout, and room for the spill step's per-body arrays (pair
// records in HBM) for the envs that take it
static int wg_a_lds_bytes(int N, int tcap) {
  const int a = wg_layout_a(N, tcap).total, s = spill::layout(N, false).total;
  return a > s ? a : s;
}
// the largest dynamic LDS of the step's kernels (checked against the device at world creation)
int wg_lds_bytes(int N, int tcap) {
  int m = wg_a_lds_bytes(N, tcap);
  if (wg_solve_lds(N) > m) m = wg_solve_lds(N);
  if (wg::wg_layout_d(N, tcap).total > m) m = wg::wg_layout_d(N, tcap).total;
  if (wg_layout_c(N).total > m) m = wg_layout_c(N).total;
  if (wg_init_lds_bytes(N) > m) m = wg_init_lds_bytes(N);
  return m;
}

// Raise the dynamic-LDS limit of the workgroup kernels (world creation). The limit is a property of
// the kernel, not of a world: it only ever grows (per device), so creating a world of fewer agents
// after a larger one cannot make the larger world's launches fail.
hipError_t wg_configure(int N, int tcap) {
  static std::mutex mu;
  static std::map<int, int> high;  // device -> the largest N configured
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  int& hw = high[dev];
  if (N <= hw) return hipSuccess;
  hw = N;
  hipError_t e = hipSuccess;
  const void* fi[] = {(const void*)flock_init_wg<float>, (const void*)flock_init_wg<double>};
  for (const void* f : fi)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, wg_init_lds_bytes(N));
  const void* fsplit[] = {(const void*)flock_step_wg_a<float>, (const void*)flock_step_wg_a<double>,
                          (const void*)flock_solve_wg, (const void*)flock_step_wg_c<float>,
                          (const void*)flock_step_wg_c<double>};
  const int la = wg_a_lds_bytes(N, tcap), lc = wg_layout_c(N).total;
  const int lsplit[] = {la, la, wg_solve_lds(N), lc, lc};
  for (int i = 0; i < 5; ++i)
    if (e == hipSuccess) e = hipFuncSetAttribute(fsplit[i], hipFuncAttributeMaxDynamicSharedMemorySize, lsplit[i]);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)flock_dfs_wg, hipFuncAttributeMaxDynamicSharedMemorySize,
                            wg::wg_layout_d(N, tcap).total);
  return e;
}

// One workgroup-path step: the env order, kernels A, DFS, B and C. With a handoff (HS non-NULL, and
// stream waits supported), kernel C runs on HS->stream as B's consumer (see Handoff): that stream
// waits for every B wave to have started, C's blocks take the envs in B's finish order, and the
// caller's stream waits for C at the end, so the call's results are complete on `s` as before.
hipError_t launch_step_wg(const StepParams& P, const WorldBuffers& B, int cur, int tcap, const void* actions,
                          void* obs, bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done,
                          hipStream_t s, HandoffStream* HS, uint8_t* bot_act) {
  dim3 grid(P.n_envs), block(wg_block(P.n_agents));
  Handoff H{nullptr, nullptr, nullptr, 0u};
  if (HS && B.sched) {
    if (++HS->tag == 0u) HS->tag = 1u;  // 0 never tags a step (zeroed queue entries)
    H = Handoff{HS->b_started, HS->ctr, HS->q, HS->tag};
  }
  if (B.sched) {
    const hipError_t oe = launch_env_order(reinterpret_cast<const uint32_t*>(B.ccount[cur]), B.sched, P.n_envs,
                                           P.max_contacts, s, H.q ? H.ctr : nullptr);
    if (oe != hipSuccess) return oe;
  }
  const int N = P.n_agents, la = wg_a_lds_bytes(N, tcap), lc = wg_layout_c(N).total;
  const int ld = wg::wg_layout_d(N, tcap).total;
  auto launch_c = [&](hipStream_t cs) {
    if (obs_f64)
      hipLaunchKernelGGL(flock_step_wg_c<double>, grid, block, lc, cs, P, B, cur, tcap, (double*)obs, nbr, rew, coll,
                         done, H, bot_act);
    else
      hipLaunchKernelGGL(flock_step_wg_c<float>, grid, block, lc, cs, P, B, cur, tcap, (float*)obs, nbr, rew, coll,
                         done, H, bot_act);
  };
  if (obs_f64)
    hipLaunchKernelGGL(flock_step_wg_a<double>, grid, block, la, s, P, B, cur, tcap, actions, (double*)obs, nbr, rew,
                       coll, done);
  else
    hipLaunchKernelGGL(flock_step_wg_a<float>, grid, block, la, s, P, B, cur, tcap, actions, (float*)obs, nbr, rew,
                       coll, done);
  // the watcher's clock starts only once kernel B's dependencies have finished: HS->stream
  // waits for this event, recorded on `s` right before B, so work queued on the caller's stream ahead
  // of the step (a policy update, another world's launches) cannot run the watcher out of time
  hipLaunchKernelGGL(flock_dfs_wg, grid, dim3(64), ld, s, P, B, tcap);
  const bool pre_b = H.q && hipEventRecord(HS->pre_b, s) == hipSuccess;
  hipLaunchKernelGGL(flock_solve_wg, grid, dim3(64), wg_solve_lds(N), s, P, B, tcap, H);
  if (!H.q) {
    launch_c(s);
    return hipGetLastError();
  }
  // C on the second stream, behind a watcher that ends once all of B has started. The count it waits
  // for follows the B launches that were accepted (every one of their waves adds itself); a watcher
  // that cannot be launched runs C on the caller's stream after B instead (it takes B's envs from
  // the complete queue).
  hipError_t e = hipPeekAtLastError();
  if (e != hipSuccess) return e;  // B not launched: nothing on the second stream, no count to wait for
  HS->expected += (unsigned long long)P.n_envs;
  if (!pre_b || hipStreamWaitEvent(HS->stream, HS->pre_b, 0) != hipSuccess ||
      launch_wait_count(HS->b_started, HS->expected, B.host_status, HS->stream) != hipSuccess) {
    (void)hipGetLastError();
    launch_c(s);
    return hipGetLastError();
  }
  launch_c(HS->stream);
  e = hipPeekAtLastError();
  // joined whatever happened above
  const hipError_t r = hipEventRecord(HS->done, HS->stream);
  const hipError_t w = hipStreamWaitEvent(s, HS->done, 0);
  if (e == hipSuccess) e = r != hipSuccess ? r : w;
  return e != hipSuccess ? e : hipGetLastError();
}

hipError_t launch_init_wg(const StepParams& P, const WorldBuffers& B, int cur, void* obs, bool obs_f64, int32_t* nbr, const uint8_t* mask,
                          hipStream_t s) {
  const int lds = wg_init_lds_bytes(P.n_agents);
  dim3 grid(P.n_envs), block(wg_block(P.n_agents));
  if (obs_f64)
    hipLaunchKernelGGL(flock_init_wg<double>, grid, block, lds, s, P, B, cur, (double*)obs, nbr, mask);
  else
    hipLaunchKernelGGL(flock_init_wg<float>, grid, block, lds, s, P, B, cur, (float*)obs, nbr, mask);
  return hipGetLastError();
}

hipError_t launch_observe_wg(const StepParams& P, const WorldBuffers& B, void* obs, bool obs_f64, int32_t* nbr,
                             hipStream_t s) {
  const int lds = 8 * P.n_agents;
  dim3 grid(P.n_envs), block(wg_block(P.n_agents));
  if (obs_f64)
    hipLaunchKernelGGL(flock_observe_wg<double>, grid, block, lds, s, P, B, (double*)obs, nbr);
  else
    hipLaunchKernelGGL(flock_observe_wg<float>, grid, block, lds, s, P, B, (float*)obs, nbr);
  return hipGetLastError();
}

}  // namespace macm
