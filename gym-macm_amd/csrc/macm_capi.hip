// macm_capi.hip — the C-ABI of libmacm_hip.so (declared in include/macm.h).
//
// Owns the per-world device state (SoA, sized for E envs x N agents), derives the
// step constants from macm_config the way the reference derives them, seeds
// envs with the reference's RNG order, and launches the HIP kernels on the
// caller's stream. No torch types, no exceptions across the ABI.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "flock_common.hpp"
#include "py_mt19937.hpp"

namespace macm {
hipError_t launch_step_w64(const StepParams& P, const WorldBuffers& B, int cur, const void* actions, void* obs,
                           bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done, hipStream_t s);
hipError_t launch_rollout_w64(const StepParams& P, const WorldBuffers& B, int cur, const void* actions, void* obs,
                              bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done, hipStream_t s,
                              int nsteps, unsigned long long astride, int traj);
hipError_t launch_init_w64(const StepParams& P, const WorldBuffers& B, int cur, void* obs, bool obs_f64,
                           int32_t* nbr, const uint8_t* mask, hipStream_t s);
hipError_t launch_observe_w64(const StepParams& P, const WorldBuffers& B, void* obs, bool obs_f64, int32_t* nbr,
                              hipStream_t s);
hipError_t launch_step_wg(const StepParams& P, const WorldBuffers& B, int cur, int tcap, const void* actions,
                          void* obs, bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done,
                          hipStream_t s, HandoffStream* HS, uint8_t* bot_act = nullptr);
hipError_t launch_init_wg(const StepParams& P, const WorldBuffers& B, int cur, void* obs, bool obs_f64, int32_t* nbr,
                          const uint8_t* mask, hipStream_t s);
hipError_t launch_observe_wg(const StepParams& P, const WorldBuffers& B, void* obs, bool obs_f64, int32_t* nbr,
                             hipStream_t s);
hipError_t launch_tdm_step_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                               const TdmBuffers& TB, int cur, const void* actions, void* obs, bool obs_f64,
                               uint8_t* done, hipStream_t s);
hipError_t launch_tdm_rollout_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                                  const TdmBuffers& TB, int cur, const void* actions, void* obs, bool obs_f64,
                                  uint8_t* done, hipStream_t s, int nsteps, unsigned long long astride, int traj,
                                  unsigned long long* tail_ctl = nullptr, unsigned tail_tag = 0u, int tail_workers = 0,
                                  int tail_k0 = 0);
int tdm_rollout_resident_blocks(int n_agents, bool obs_f64);
hipError_t launch_tdm_init_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                               const TdmBuffers& TB, int cur, void* obs, bool obs_f64, const uint8_t* mask,
                               hipStream_t s);
hipError_t launch_draw_poses(const uint8_t* mask, uint32_t* mt, const PoseDraw& D, int n_envs, float2* pos,
                             float* angle, hipStream_t s);
hipError_t launch_tdm_step_wg(const StepParams& P, const WorldBuffers& B, const TdmParams& TP, const TdmBuffers& TB,
                              int cur, const void* actions, void* obs, bool obs_f64, uint8_t* done, hipStream_t s);
hipError_t launch_tdm_init_wg(const StepParams& P, const WorldBuffers& B, const TdmParams& TP, const TdmBuffers& TB,
                              int cur, void* obs, bool obs_f64, const uint8_t* mask, hipStream_t s);
hipError_t launch_tdm_observe_wg(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                                 const TdmBuffers& TB, void* obs, bool obs_f64, hipStream_t s);
hipError_t launch_tdm_observe_snap(const TdmParams& TP, int N, size_t rows, const float4* snap, void* obs,
                                   bool obs_f64, uint8_t* mask, hipStream_t s);
hipError_t tdm_wg_configure(int N);
int tdm_wg_step_lds(int N);
int tdm_wg_obs_lds(int N);
hipError_t launch_tdm_observe_w64(const StepParams& P, const WorldBuffers& B, const TdmParams& TP,
                                  const TdmBuffers& TB, void* obs, bool obs_f64, hipStream_t s);
hipError_t launch_bots_flock(const void* obs, bool obs_f64, int od, long long rows, uint8_t* act, hipStream_t s);
hipError_t launch_bots_combat(const void* obs, const uint8_t* mask, bool obs_f64, int N, long long rows,
                              uint8_t* act, hipStream_t s);
hipError_t wg_configure(int N, int tcap);
// worlds of 1024 < N <= 4096 agents (flock_big.hip)
hipError_t big_configure(int N);
int big_step_lds(int N);
int big_init_lds(int N);
hipError_t launch_step_big(const StepParams& P, const WorldBuffers& B, int cur, const void* actions, void* obs,
                           bool obs_f64, int32_t* nbr, float* rew, uint8_t* coll, uint8_t* done, hipStream_t s);
hipError_t launch_init_big(const StepParams& P, const WorldBuffers& B, int cur, void* obs, bool obs_f64, int32_t* nbr,
                           const uint8_t* mask, hipStream_t s);
hipError_t launch_observe_big(const StepParams& P, const WorldBuffers& B, void* obs, bool obs_f64, int32_t* nbr,
                              hipStream_t s);
int wg_block(int N);
int wg_lds_bytes(int N, int tcap);
hipError_t launch_check_actions(const void* actions, int mode, const uint8_t* alive, long long rows,
                                unsigned long long* first_bad, hipStream_t s);
hipError_t launch_check_lists(const int32_t* count, const uint32_t* ab, int E, int C, int cap, int N,
                              unsigned long long* first_bad, hipStream_t s);
}  // namespace macm

using namespace macm;

struct macm_world {
  macm_config cfg;
  StepParams P;
  WorldBuffers B;
  int cur;  // which contact-list buffer holds the current ordered list
  int device;
  bool wave;  // N <= 64: one wavefront per env (flock_step_w64); else one workgroup per env
  bool big;   // N > 1024: the spill step with several bodies per thread (flock_big.hip)
  int tcap;   // touching-contact capacity per env of the fast kernels (more: the spill step)
  std::vector<int32_t> tidx;
  std::vector<void*> allocs;
  uint32_t* mt = nullptr;     // [E][kMtStride] per-env MT19937 streams (valid after reset)
  uint8_t* rmask = nullptr;   // [E] reset mask scratch
  bool mt_valid = false;
  uint32_t* hstat = nullptr;  // host-mapped status word (B.host_status is its device alias)
  unsigned long long* bad = nullptr;  // validate_actions: first failing row (device scratch)
  // workgroup-path rollouts: env slices on streams of their own (created on first use)
  std::vector<hipStream_t> slice_streams;
  std::vector<hipEvent_t> slice_events;  // [0] fork, [1 + s] join of slice s
  HandoffStream* ho = nullptr;  // workgroup path: kernel C as kernel B's consumer (handoff_for)
  bool ho_tried = false;
  int slots_alloc = 0;  // spill working-set slots allocated (== E: one per env)
  int pool0 = 0;        // B.sp_pool as created (0: one slot per env), restored by set_debug
};

struct macm_tdm {
  macm_tdm_config cfg;
  StepParams P;
  WorldBuffers B;
  TdmParams TP;
  TdmBuffers TB;  // state pointers; output pointers are filled per call
  int cur;
  int device;
  bool wave;  // N <= 64: the wave kernel (env_step_w64<kTdm>); else the workgroup step (tdm_step_wg.hip)
  std::vector<int> team;  // agent -> team
  std::vector<void*> allocs;
  uint32_t* mt = nullptr;
  uint8_t* rmask = nullptr;
  bool mt_valid = false;
  uint32_t* hstat = nullptr;
  unsigned long long* bad = nullptr;
  int slots_alloc = 0;  // as macm_world
  int pool0 = 0;
  // the split observation (tdm_obs_snap.hip, tdm_split_obs): pose snapshots in two halves of
  // snap_rows (step, env) rows each, the observation stream and the chunk events (created on first use)
  float4* snap = nullptr;
  size_t snap_rows = 0;
  hipStream_t obs_stream = nullptr;
  hipEvent_t ev_phys[2] = {nullptr, nullptr}, ev_obs[2] = {nullptr, nullptr};
  // the tail observation (flock_step_w64.hip TailObs, tdm_tail_obs): snapshots of every (step, env)
  // row of a rollout, the row counters and ready words, the last launch's tag, the resident capacity
  float4* tail_snap = nullptr;
  size_t tail_rows = 0;
  unsigned long long* tail_ctl = nullptr;
  unsigned tail_tag = 0;
  int tail_cap = -1;
};

static thread_local std::string g_last_error;

static int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return fail(MACM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));             \
  } while (0)

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <typename T>
int dalloc(std::vector<void*>& allocs, T** p, size_t count) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, count * sizeof(T) > 0 ? count * sizeof(T) : 16);
  if (e != hipSuccess) return fail(MACM_E_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
  allocs.push_back(q);
  *p = (T*)q;
  return MACM_OK;
}

template <typename T>
int dalloc(macm_world* w, T** p, size_t count) {
  return dalloc(w->allocs, p, count);
}

int obs_dim(const macm_config& c) { return c.coord == MACM_COORD_CARTESIAN ? 6 : 4; }

// Step constants shared by Flock and TDM, derived as the reference derives them.
void fill_body_params(StepParams& P, double hz, float radius, float density, float friction, float damping,
                      double agent_force, double rotation_speed) {
  // cm_framework.py:182-185 (timeStep = 1.0 / hz, a Python float) -> b2World::Step(float32 dt)
  volatile double dt64 = 1.0 / hz;
  P.dt = (float)dt64;
  P.inv_dt = 1.0f / P.dt;
  {
    // b2CircleShape::ComputeMass + b2Body::ResetMassData (settings.py:127-133)
    volatile float mass = density * kPi32 * radius * radius;
    P.inv_mass = mass > 0.0f ? 1.0f / mass : 1.0f;
    volatile float den = 1.0f + P.dt * damping;
    P.damp = 1.0f / den;
    volatile float ff = friction * friction;
    P.friction = sqrtf(ff);  // b2MixFriction
  }
  P.radius = radius;
  P.force_f32 = (float)agent_force;
  P.rot_step = rotation_speed;
  P.inv_hz = 1.0 / hz;
  P.force = agent_force;
  volatile double two = 2.0;
  P.diag_c = 1.0 / sqrt(two);  // 1 / np.sqrt(2)
}

static void free_handoff(HandoffStream*& h) {
  if (!h) return;
  if (h->stream) (void)hipStreamDestroy(h->stream);
  if (h->done) (void)hipEventDestroy(h->done);
  if (h->pre_b) (void)hipEventDestroy(h->pre_b);
  if (h->b_started) (void)hipFree(h->b_started);
  if (h->ctr) (void)hipFree(h->ctr);
  if (h->q) (void)hipFree(h->q);
  delete h;
  h = nullptr;
}

void free_world(macm_world* w) {
  free_handoff(w->ho);
  for (hipStream_t st : w->slice_streams) (void)hipStreamDestroy(st);
  for (hipEvent_t ev : w->slice_events) (void)hipEventDestroy(ev);
  w->slice_streams.clear();
  w->slice_events.clear();
  for (void* p : w->allocs) (void)hipFree(p);
  w->allocs.clear();
  if (w->hstat) (void)hipHostFree(w->hstat);
  w->hstat = nullptr;
}

// The host-mapped status word: kernels store nonzero status bits into it (report_status), and
// the step entry points read it without synchronising. Returns its device alias.
hipError_t alloc_host_status(uint32_t** host, uint32_t** dev) {
  hipError_t e = hipHostMalloc((void**)host, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return e;
  **host = 0u;
  return hipHostGetDevicePointer((void**)dev, *host, 0);
}

uint32_t read_host_status(const uint32_t* h) { return h ? __atomic_load_n(h, __ATOMIC_ACQUIRE) : 0u; }
void clear_host_status(uint32_t* h) {
  if (h) __atomic_store_n(h, 0u, __ATOMIC_RELEASE);
}

// After reset_envs: the init kernel rewrote the reset envs' status, so a set host word becomes the OR
// of what the envs still carry (0 once every overflowed env was reset; ADVICE r02: it kept the stale
// bits, and every later step failed). Only then does it synchronise the stream: with the word clear
// (the normal case, e.g. autoreset every step) reset_envs stays asynchronous.
int resync_host_status(uint32_t* h, const int32_t* dev_status, int E, hipStream_t s) {
  if (read_host_status(h) == 0u) return MACM_OK;
  std::vector<int32_t> st(E);
  HIP_TRY(hipMemcpyAsync(st.data(), dev_status, E * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  uint32_t acc = 0u;
  for (int32_t v : st) acc |= (uint32_t)v;
  if (h) __atomic_store_n(h, acc, __ATOMIC_RELEASE);
  return MACM_OK;
}

// Default capacities (macm_world_create in include/macm.h), from a per-world memory budget of
// 1/8 of the device's free memory at creation (a fixed 8 GiB per world multiplied with
// the worlds or ranks sharing a device; every world now shrinks what the next one sees), half for
// the contact lists, half for the spill step's working set:
//   C = every pair when E * C * 24 B (two lists of pair + impulses) fits the lists' half (always
//       for N <= 64, the wave kernel), else the largest such C (at least 32 N);
//   S = spill working-set slots of 48 B per entry (C entries) + 48 B per body: one per env when
//       they fit the other half, else as many as fit (at least 16), taken by spilling envs in turn.
struct Capacity {
  int64_t C;
  int64_t slots;  // == E: one slot per env
};
// Kernel dispatches run one at a time: HIP's serialisation switches, or a profiler collecting counters
// (rocprofv3 --pmc serialises dispatches to attribute counters to them). The producer/consumer
// launch pair of the B -> C handoff needs its consumer to run BESIDE the producer: under
// serialisation the consumer's wait would time out and the step be left incomplete, so it is off.
static bool serialized_dispatch() {
  for (const char* k : {"AMD_SERIALIZE_KERNEL", "HIP_LAUNCH_BLOCKING", "CUDA_LAUNCH_BLOCKING"}) {
    const char* v = getenv(k);
    if (v && atoi(v) != 0) return true;
  }
  const char* pmc = getenv("ROCPROF_COUNTER_COLLECTION");
  return pmc && *pmc && strcmp(pmc, "0") != 0 && strcasecmp(pmc, "false") != 0;
}

// The most agents per env (Flock and TDM): one workgroup of 1024 threads, up to 4 bodies per thread
// (flock_big.hip, the spill step's BPT), 16-bit body ids in the lists (b < 32768 with a flag bit)
constexpr int kMaxAgents = 4096;

Capacity default_capacity(int N, int E, int64_t max_contacts, size_t free_bytes) {
  const int64_t all_pairs = (int64_t)N * (N - 1) / 2;
  const int64_t budget = std::max<int64_t>((int64_t)(free_bytes / 8), 256LL << 20);
  const int64_t half = budget / 2;
  Capacity cap;
  if (max_contacts > 0) cap.C = max_contacts;
  else if (N <= 64 || all_pairs * 24 * E <= half) cap.C = all_pairs;
  else cap.C = std::max<int64_t>(32LL * N, half / (24LL * E));
  cap.C = std::max<int64_t>(1, std::min(cap.C, all_pairs));
  const int64_t per_slot = cap.C * 48 + (int64_t)N * 48;
  cap.slots = std::min<int64_t>(E, std::max<int64_t>(16, half / per_slot));
  return cap;
}

// validate_actions (macm_config / macm_tdm_config): run the check kernel and wait for it.
// rows = n_steps * n_envs for a rollout's [K, E, N, A] actions; n_envs decodes the offending row
// into (step, env) (the env was reported as step * E + env)
int check_actions(unsigned long long* bad, const void* actions, int mode, const uint8_t* alive, int E, int N,
                  hipStream_t s, int n_envs = 0) {
  HIP_TRY(hipMemsetAsync(bad, 0xff, sizeof(unsigned long long), s));
  HIP_TRY(launch_check_actions(actions, mode, alive, (long long)E * N, bad, s));
  unsigned long long h = ~0ull;
  HIP_TRY(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (h != ~0ull) {
    const char* space = mode == 0 ? "MultiDiscrete([3, 3, 3])" : mode == 1 ? "Box([-1, -1], [1, 1])"
                                                                           : "MultiDiscrete([3, 3, 3, 2])";
    const unsigned long long row = h / N;
    const std::string where = n_envs > 0 && (unsigned long long)E > (unsigned long long)n_envs
                                  ? "step " + std::to_string(row / n_envs) + " env " + std::to_string(row % n_envs)
                                  : "env " + std::to_string(row);
    return fail(MACM_E_INVALID, "action of " + where + " agent " + std::to_string(h % N) +
                                    " is not in the action space " + space + " (no env was stepped)");
  }
  return MACM_OK;
}

hipError_t launch_init(macm_world* w, const macm_outputs* out, const uint8_t* mask, hipStream_t s) {
  void* obs = out ? out->obs : nullptr;
  int32_t* nbr = out ? out->nbr_id : nullptr;
  if (w->wave) return launch_init_w64(w->P, w->B, w->cur, obs, w->cfg.obs_f64 != 0, nbr, mask, s);
  if (w->big) return launch_init_big(w->P, w->B, w->cur, obs, w->cfg.obs_f64 != 0, nbr, mask, s);
  return launch_init_wg(w->P, w->B, w->cur, obs, w->cfg.obs_f64 != 0, nbr, mask, s);
}

// Host generator state -> the env's slot of the device stream buffer.
void save_stream(std::vector<uint32_t>& host, int e, const PyMT19937& r) {
  uint32_t* d = host.data() + (size_t)e * kMtStride;
  memcpy(d, r.state(), sizeof(uint32_t) * PyMT19937::kWords);
  d[PyMT19937::kWords] = (uint32_t)r.index();
}

}  // namespace

extern "C" {

const char* macm_version(void) {
  return "macm-hip 0.6.0 (gfx950; Flock: wave-per-env kernel N<=64, workgroup-per-env kernels N<=1024, "
         "spill step for dense envs and N<=4096; TDM: wave-per-env kernel N<=64, workgroup step N<=4096)";
}
int macm_abi_version(void) { return MACM_ABI_VERSION; }
const char* macm_last_error(void) { return g_last_error.c_str(); }

int macm_config_default(macm_config* c) {
  if (!c) return fail(MACM_E_INVALID, "cfg is NULL");
  memset(c, 0, sizeof(*c));
  c->n_agents = 10;  // Flock(n_agents=[10]) default, mvmnt.py:35
  c->n_targets = 1;
  c->action_mode = MACM_ACTION_DISCRETE;
  c->reward_mode = MACM_REWARD_BINARY;
  c->coord = MACM_COORD_POLAR;
  c->velocity_iterations = 8;
  c->position_iterations = 3;
  c->warm_starting = 1;
  c->obs_f64 = 0;
  c->hz = 60.0;
  c->start_spread = 20.0;
  c->start_point[0] = 0.0;
  c->start_point[1] = 0.0;
  c->agent_rotation_speed = 0.8 * (2 * M_PI);
  c->agent_force = 20.0;
  c->time_limit = 60.0;
  c->reward_radius = 7.0;
  c->target_mindist = 25.0;
  c->target_maxdist = 60.0;
  c->radius = 0.5f;
  c->density = 1.0f;
  c->friction = 0.3f;
  c->linear_damping = 5.0f;
  return MACM_OK;
}

int macm_world_create(const macm_config* cfg, const int32_t* targets_idx, int32_t n_envs, int32_t device,
                      int32_t max_contacts, macm_world** out) {
  if (!cfg || !out) return fail(MACM_E_INVALID, "cfg/out is NULL");
  *out = nullptr;
  const macm_config& c = *cfg;
  if (n_envs <= 0) return fail(MACM_E_INVALID, "n_envs must be > 0");
  if (c.n_agents < 2) return fail(MACM_E_INVALID, "n_agents must be >= 2 (get_obs needs another agent)");
  if (c.n_agents > kMaxAgents)
    return fail(MACM_E_UNSUPPORTED, "n_agents > 4096 is not built (one workgroup per env, <= 4 bodies per thread)");
  if (c.n_targets < 1) return fail(MACM_E_INVALID, "n_targets must be >= 1");
  if (!(c.hz > 0.0)) return fail(MACM_E_INVALID, "hz must be > 0");
  if (c.velocity_iterations < 0 || c.position_iterations < 0) return fail(MACM_E_INVALID, "iterations < 0");
  if (c.action_mode != MACM_ACTION_DISCRETE && c.action_mode != MACM_ACTION_CONTINUOUS)
    return fail(MACM_E_INVALID, "action_mode");
  if (c.reward_mode != MACM_REWARD_BINARY && c.reward_mode != MACM_REWARD_LINEAR)
    return fail(MACM_E_INVALID, "reward_mode");
  if (c.coord != MACM_COORD_POLAR && c.coord != MACM_COORD_CARTESIAN) return fail(MACM_E_INVALID, "coord");
  if (!(c.radius > 0.0f)) return fail(MACM_E_INVALID, "radius must be > 0");
  const int N = c.n_agents, T = c.n_targets;
  std::vector<int32_t> tidx(N, 0);
  if (targets_idx)
    for (int i = 0; i < N; ++i) {
      if (targets_idx[i] < 0 || targets_idx[i] >= T) return fail(MACM_E_INVALID, "targets_idx out of range");
      tidx[i] = targets_idx[i];
    }
  if (max_contacts < 0) return fail(MACM_E_INVALID, "max_contacts must be >= 0");

  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MACM_E_INVALID, "device index out of range");
  DeviceGuard g(device);
  size_t free_bytes = 0, total_bytes = 0;
  HIP_TRY(hipMemGetInfo(&free_bytes, &total_bytes));
  const Capacity cap = default_capacity(N, n_envs, max_contacts, free_bytes);
  const int C = (int)cap.C;
  const int64_t SL = cap.slots;  // spill working-set slots

  macm_world* w = new macm_world();
  w->cfg = c;
  w->device = device;
  w->cur = 0;
  w->tidx = tidx;
  w->wave = N <= 64;
  w->big = N > 1024;  // flock_big.hip: the spill step with several bodies per thread
  {
    const int bs = N <= 64 ? 64 : wg_block(N);
    const int want = N <= 64 ? 256 : 5 * bs;  // register staging holds 5 records per thread
    w->tcap = w->big ? C : want < 4608 ? want : 4608;  // big: every touching contact takes the spill step
  }
  StepParams& P = w->P;
  P.n_envs = n_envs;
  P.n_agents = N;
  P.n_targets = T;
  P.max_contacts = C;
  P.vel_iters = c.velocity_iterations;
  P.pos_iters = c.position_iterations;
  P.warm_starting = c.warm_starting ? 1 : 0;
  P.action_mode = c.action_mode;
  P.reward_mode = c.reward_mode;
  P.coord = c.coord;
  P.force_spill = 0;
  P.sweep = 0;
  fill_body_params(P, c.hz, c.radius, c.density, c.friction, c.linear_damping, c.agent_force,
                   c.agent_rotation_speed);
  P.reward_radius = c.reward_radius;
  P.time_limit = c.time_limit;

  WorldBuffers& B = w->B;
  memset(&B, 0, sizeof(B));
  const size_t EN = (size_t)n_envs * N;
  int rc = MACM_OK;
  if ((rc = dalloc(w, &B.pos, EN)) || (rc = dalloc(w, &B.vel, EN)) || (rc = dalloc(w, &B.angle, EN)) ||
      (rc = dalloc(w, &B.fat, EN)) || (rc = dalloc(w, &B.sleep, EN)) ||
      (rc = dalloc(w, &B.targets, (size_t)n_envs * T)) || (rc = dalloc(w, &B.tidx, (size_t)N)) ||
      (rc = dalloc(w, &B.ccount[0], (size_t)n_envs)) || (rc = dalloc(w, &B.ccount[1], (size_t)n_envs)) ||
      (rc = dalloc(w, &B.cab[0], (size_t)n_envs * C)) || (rc = dalloc(w, &B.cab[1], (size_t)n_envs * C)) ||
      (rc = dalloc(w, &B.cimp[0], (size_t)n_envs * C)) || (rc = dalloc(w, &B.cimp[1], (size_t)n_envs * C)) ||
      (rc = dalloc(w, &B.step_count, (size_t)n_envs)) || (rc = dalloc(w, &B.time_passed, (size_t)n_envs)) ||
      (rc = dalloc(w, &B.done, (size_t)n_envs)) || (rc = dalloc(w, &B.status, (size_t)n_envs)) ||
      (rc = dalloc(w, &B.env_counters, (size_t)n_envs * 4)) || (rc = dalloc(w, &B.env_rsum, (size_t)n_envs))
#ifdef MACM_STAMPS
      || (rc = dalloc(w, &B.stamps, (size_t)n_envs * 32))
#endif
      || (!w->wave && !w->big && (rc = dalloc(w, &B.scratch, (size_t)n_envs * w->tcap))) ||
      (!w->wave && !w->big && ((rc = dalloc(w, &B.x_cst, (size_t)n_envs * w->tcap)) ||
                    (rc = dalloc(w, &B.x_cimp, (size_t)n_envs * w->tcap)) ||
                    (rc = dalloc(w, &B.x_ord, (size_t)n_envs * w->tcap)) ||
                    (rc = dalloc(w, &B.x_ic, (size_t)n_envs * (N / 2 + 2))) ||
                    (rc = dalloc(w, &B.x_nlvl, (size_t)n_envs)) ||
                    (rc = dalloc(w, &B.x_ib, (size_t)n_envs * (N / 2 + 2))) ||
                    (rc = dalloc(w, &B.x_ibod, EN)) || (rc = dalloc(w, &B.x_nisl, (size_t)n_envs)) ||
                    (rc = dalloc(w, &B.x_vmid, EN)) || (rc = dalloc(w, &B.x_cout, EN)) ||
                    (rc = dalloc(w, &B.x_vout, EN)) || (rc = dalloc(w, &B.x_deg, EN)) ||
                    (rc = dalloc(w, &B.x_isolv, (size_t)n_envs * (N / 2 + 2))) ||
                    (rc = dalloc(w, &B.x_tab, (size_t)n_envs * w->tcap)) ||
                    (rc = dalloc(w, &B.x_adj, (size_t)n_envs * 2 * w->tcap)) ||
                    (rc = dalloc(w, &B.x_off, (size_t)n_envs * (N + 1))) ||
                    (rc = dalloc(w, &B.x_dfs, (size_t)n_envs * w->tcap)))) ||
      // spill step working set (flock_spill.hpp), capacity C per slot, SL slots
      (rc = dalloc(w, &B.sp_tab, (size_t)SL * C)) || (rc = dalloc(w, &B.sp_adj, (size_t)SL * 2 * C)) ||
      (rc = dalloc(w, &B.sp_ord, (size_t)SL * C)) || (rc = dalloc(w, &B.sp_cst, (size_t)SL * C)) ||
      (rc = dalloc(w, &B.sp_cim, (size_t)SL * C)) || (rc = dalloc(w, &B.sp_lam, (size_t)SL * C)) ||
      (!w->wave && (rc = dalloc(w, (float4**)&B.sp_rec, (size_t)SL * N * 3))) ||  // 48-B records
      (SL < n_envs && (rc = dalloc(w, &B.sp_lock, (size_t)SL))) ||
      (rc = dalloc(w, &B.spill_count, (size_t)n_envs)) || (rc = dalloc(w, &w->bad, 1)) ||
      (rc = dalloc(w, &B.sched, (size_t)n_envs)) ||
      (rc = dalloc(w, &w->mt, (size_t)n_envs * kMtStride)) || (rc = dalloc(w, &w->rmask, (size_t)n_envs))
  ) {
    free_world(w);
    delete w;
    return rc;
  }
  if (hipError_t he = alloc_host_status(&w->hstat, &B.host_status); he != hipSuccess) {
    free_world(w);
    delete w;
    return fail(MACM_E_OOM, std::string("hipHostMalloc (status word): ") + hipGetErrorString(he));
  }
  hipError_t e = hipMemcpy(B.tidx, tidx.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(B.env_counters, 0, (size_t)n_envs * 4 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(B.env_rsum, 0, (size_t)n_envs * sizeof(double));
  if (e == hipSuccess) e = hipMemset(B.ccount[0], 0, sizeof(int32_t) * n_envs);
  if (e == hipSuccess) e = hipMemset(B.status, 0, sizeof(int32_t) * n_envs);
  if (e == hipSuccess) e = hipMemset(B.spill_count, 0, sizeof(uint32_t) * n_envs);
  B.sp_pool = SL < n_envs ? (int32_t)SL : 0;
  w->slots_alloc = (int)SL;
  w->pool0 = B.sp_pool;
  if (e == hipSuccess && B.sp_lock) e = hipMemset(B.sp_lock, 0, sizeof(uint32_t) * SL);
  if (e == hipSuccess && w->big) {
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e == hipSuccess && (size_t)std::max(big_step_lds(N), big_init_lds(N)) > prop.sharedMemPerBlock) {
      free_world(w);
      delete w;
      return fail(MACM_E_UNSUPPORTED, "per-env LDS layout exceeds the device's LDS per workgroup");
    }
    if (e == hipSuccess) e = big_configure(N);
  } else if (e == hipSuccess && !w->wave) {
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e == hipSuccess && (size_t)wg_lds_bytes(N, w->tcap) > prop.sharedMemPerBlock) {
      free_world(w);
      delete w;
      return fail(MACM_E_UNSUPPORTED, "per-env LDS layout exceeds the device's LDS per workgroup");
    }
    if (e == hipSuccess) e = wg_configure(N, w->tcap);
  }
  if (e != hipSuccess) {
    free_world(w);
    delete w;
    return fail(MACM_E_HIP, std::string("world init copy: ") + hipGetErrorString(e));
  }
  *out = w;
  return MACM_OK;
}

int macm_world_destroy(macm_world* w) {
  if (!w) return MACM_OK;
  DeviceGuard g(w->device);
  (void)hipDeviceSynchronize();
  free_world(w);
  delete w;
  return MACM_OK;
}

static int wg_rollout_slices(const macm_world* w);

int macm_world_info_get(const macm_world* w, macm_world_info* info) {
  if (!w || !info) return fail(MACM_E_INVALID, "NULL argument");
  info->n_envs = w->P.n_envs;
  info->n_agents = w->P.n_agents;
  info->n_targets = w->P.n_targets;
  info->obs_dim = obs_dim(w->cfg);
  info->max_contacts = w->P.max_contacts;
  info->max_touching = w->tcap;
  info->device = w->device;
  info->spill_slots = w->B.sp_pool > 0 ? w->B.sp_pool : w->P.n_envs;
  info->launch_flags = w->ho ? MACM_LAUNCH_HANDOFF : 0;
  info->rollout_slices = wg_rollout_slices(w);
  return MACM_OK;
}

int macm_world_reset(macm_world* w, uint64_t seed, int64_t env_offset, const macm_outputs* out, void* stream) {
  if (!w) return fail(MACM_E_INVALID, "world is NULL");
  DeviceGuard g(w->device);
  const macm_config& c = w->cfg;
  const int E = w->P.n_envs, N = w->P.n_agents, T = w->P.n_targets;
  std::vector<float2> pos((size_t)E * N), tg((size_t)E * T);
  std::vector<float> ang((size_t)E * N);
  std::vector<uint32_t> mts((size_t)E * kMtStride);
  for (int e = 0; e < E; ++e) {
    PyMT19937 r(seed + (uint64_t)(env_offset + e));
    for (int t = 0; t < T; ++t) {  // mvmnt.py:46-52
      const double rand_angle = 2 * M_PI * r.random();
      const double rand_dist = c.target_mindist + r.random() * (c.target_maxdist - c.target_mindist);
      tg[(size_t)e * T + t] = make_float2((float)(rand_dist * cos(rand_angle)), (float)(rand_dist * sin(rand_angle)));
    }
    for (int i = 0; i < N; ++i) {  // mvmnt.py:61-64, CreateDynamicBody(position=(x, y), angle=angle)
      const double x = c.start_spread * (r.random() - 0.5) + c.start_point[0];
      const double y = c.start_spread * (r.random() - 0.5) + c.start_point[1];
      const double a = r.uniform(-1, 1) * M_PI;
      pos[(size_t)e * N + i] = make_float2((float)x, (float)y);
      ang[(size_t)e * N + i] = (float)a;
    }
    save_stream(mts, e, r);
  }
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipStreamSynchronize(s));  // earlier steps' status stores land before the word is cleared
  clear_host_status(w->hstat);
  HIP_TRY(hipMemcpyAsync(w->B.pos, pos.data(), pos.size() * sizeof(float2), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(w->B.angle, ang.data(), ang.size() * sizeof(float), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(w->B.targets, tg.data(), tg.size() * sizeof(float2), hipMemcpyHostToDevice, s));
  w->cur = 0;
  HIP_TRY(hipMemcpyAsync(w->mt, mts.data(), mts.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  w->mt_valid = true;
  HIP_TRY(launch_init(w, out, nullptr, s));
  // host vectors are read by the async copies: wait before they go out of scope
  HIP_TRY(hipStreamSynchronize(s));
  return MACM_OK;
}

int macm_world_place(macm_world* w, const void* pos, const void* angle, const void* targets,
                     const macm_outputs* out, void* stream) {
  if (!w || !pos || !angle || !targets) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  const size_t EN = (size_t)w->P.n_envs * w->P.n_agents, ET = (size_t)w->P.n_envs * w->P.n_targets;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipStreamSynchronize(s));
  clear_host_status(w->hstat);
  HIP_TRY(hipMemcpyAsync(w->B.pos, pos, EN * sizeof(float2), hipMemcpyDefault, s));
  HIP_TRY(hipMemcpyAsync(w->B.angle, angle, EN * sizeof(float), hipMemcpyDefault, s));
  HIP_TRY(hipMemcpyAsync(w->B.targets, targets, ET * sizeof(float2), hipMemcpyDefault, s));
  w->cur = 0;
  w->mt_valid = false;  // poses came from the caller's generator
  HIP_TRY(launch_init(w, out, nullptr, s));
  HIP_TRY(hipStreamSynchronize(s));
  return MACM_OK;
}

static int fill_reset_mask(uint8_t* rmask, const uint8_t* env_mask, int E, hipStream_t s) {
  // a private copy: the init kernels clear the done flags a caller may pass as the mask
  if (env_mask) HIP_TRY(hipMemcpyAsync(rmask, env_mask, (size_t)E, hipMemcpyDefault, s));
  else HIP_TRY(hipMemsetAsync(rmask, 1, (size_t)E, s));
  return MACM_OK;
}

int macm_world_reset_envs(macm_world* w, const uint8_t* env_mask, const macm_outputs* out, void* stream) {
  if (!w) return fail(MACM_E_INVALID, "world is NULL");
  if (!w->mt_valid)
    return fail(MACM_E_INVALID, "no per-env random streams: the world was placed, not reset (macm_world_reset)");
  DeviceGuard g(w->device);
  hipStream_t s = (hipStream_t)stream;
  int rc = fill_reset_mask(w->rmask, env_mask, w->P.n_envs, s);
  if (rc) return rc;
  PoseDraw D;
  memset(&D, 0, sizeof(D));
  D.mode = kFlock;
  D.n_agents = w->P.n_agents;
  D.spread = w->cfg.start_spread;
  D.start_x = w->cfg.start_point[0];
  D.start_y = w->cfg.start_point[1];
  HIP_TRY(launch_draw_poses(w->rmask, w->mt, D, w->P.n_envs, w->B.pos, w->B.angle, s));
  HIP_TRY(launch_init(w, out, w->rmask, s));
  return resync_host_status(w->hstat, w->B.status, w->P.n_envs, s);
}

static int overflow_error(uint32_t st) {
  std::string what;
  if (st & MACM_ST_CONTACT_OVERFLOW) what += " contact-list capacity (max_contacts);";
  if (st & MACM_ST_TOUCH_OVERFLOW) what += " touching-contact capacity;";
  if (st & MACM_ST_DEGREE_OVERFLOW) what += " per-body contact capacity;";
  if (st & MACM_ST_SPILL_WAIT) what += " spill working-set pool (a dense env waited ~1 s for a slot);";
  if (st & MACM_ST_HANDOFF) what += " B -> C handoff (kernel B's waves did not all start, or a kernel-C block found no env, within ~1 s; every "
                                        "env is marked: rebuild the world or reset it);";
  return fail(MACM_E_OVERFLOW, "an env outgrew its" + what +
                                   " the results since that step are not the reference's (status bits " +
                                   std::to_string(st) + "; reset, place or set_state clears them)");
}

// The workgroup step's B -> C handoff (flock_common.hpp Handoff), created at the first step that can
// use it: the workgroup path, when kHandoffDefault or MACM_HANDOFF=1 (A/B; MACM_HANDOFF=0 off). Env
// slices (rollout_wg_slices) run without it. NULL: kernel C launched after B on the same stream.
static constexpr bool kHandoffDefault = true;  // round 5: C5 window 5.35 -> 4.99 ms (profiles/r05/abtests/handoff_fused/)
static HandoffStream* handoff_for(macm_world* w) {
  if (w->wave || w->big || w->ho_tried) return w->ho;
  w->ho_tried = true;
  const char* v = getenv("MACM_HANDOFF");
  if (!(v ? atoi(v) != 0 : kHandoffDefault) || serialized_dispatch()) return nullptr;
  HandoffStream* h = new HandoffStream{};
  bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&h->done, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&h->pre_b, hipEventDisableTiming) == hipSuccess &&
            hipMalloc(&h->b_started, sizeof(unsigned long long)) == hipSuccess &&
            hipMalloc(&h->ctr, 2 * sizeof(unsigned int)) == hipSuccess &&
            hipMalloc(&h->q, (size_t)w->P.n_envs * sizeof(unsigned long long)) == hipSuccess;
  // tags start at 1, so a zeroed queue holds no entry of any step; the start count from 0
  ok = ok && hipMemset(h->q, 0, (size_t)w->P.n_envs * sizeof(unsigned long long)) == hipSuccess &&
       hipMemset(h->ctr, 0, 2 * sizeof(unsigned int)) == hipSuccess &&
       hipMemset(h->b_started, 0, sizeof(unsigned long long)) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    free_handoff(h);
    return nullptr;
  }
  w->ho = h;
  return h;
}

int macm_world_step(macm_world* w, const void* actions, const macm_outputs* out, void* stream) {
  if (!w || !actions || !out || !out->reward) return fail(MACM_E_INVALID, "world/actions/out/reward is NULL");
  if (const uint32_t st = read_host_status(w->hstat)) return overflow_error(st);
  DeviceGuard g(w->device);
  if (w->cfg.validate_actions) {
    const int rc = check_actions(w->bad, actions, w->cfg.action_mode == MACM_ACTION_DISCRETE ? 0 : 1, nullptr,
                                 w->P.n_envs, w->P.n_agents, (hipStream_t)stream);
    if (rc) return rc;
  }
  if (w->wave)
    HIP_TRY(launch_step_w64(w->P, w->B, w->cur, actions, out->obs, w->cfg.obs_f64 != 0, out->nbr_id, out->reward,
                            out->collided, out->done, (hipStream_t)stream));
  else if (w->big)
    HIP_TRY(launch_step_big(w->P, w->B, w->cur, actions, out->obs, w->cfg.obs_f64 != 0, out->nbr_id, out->reward,
                            out->collided, out->done, (hipStream_t)stream));
  else
    HIP_TRY(launch_step_wg(w->P, w->B, w->cur, w->tcap, actions, out->obs, w->cfg.obs_f64 != 0, out->nbr_id,
                           out->reward, out->collided, out->done, (hipStream_t)stream, handoff_for(w)));
  w->cur ^= 1;
  return MACM_OK;
}

// Envs [e0, e0 + n) of a world as a world of n envs: every per-env array offset by e0 rows
// (the sizes macm_world_create allocates), tidx and the status word shared.
static WorldBuffers slice_buffers(const WorldBuffers& B, size_t e0, size_t N, size_t T, size_t C, size_t tcap) {
  WorldBuffers S = B;
  const size_t EN = e0 * N, IS = e0 * (N / 2 + 2);
  auto off = [](auto*& p, size_t n) {
    if (p) p += n;
  };
  off(S.pos, EN), off(S.vel, EN), off(S.angle, EN), off(S.fat, EN), off(S.sleep, EN);
  off(S.targets, e0 * T);
  for (int c = 0; c < 2; ++c) off(S.ccount[c], e0), off(S.cab[c], e0 * C), off(S.cimp[c], e0 * C);
  off(S.step_count, e0), off(S.time_passed, e0), off(S.done, e0), off(S.status, e0);
  off(S.env_counters, e0 * 4), off(S.env_rsum, e0), off(S.stamps, e0 * 32);
  off(S.scratch, e0 * tcap), off(S.x_cst, e0 * tcap), off(S.x_cimp, e0 * tcap), off(S.x_ord, e0 * tcap);
  off(S.x_ic, IS), off(S.x_nlvl, e0), off(S.x_ib, IS), off(S.x_ibod, EN), off(S.x_nisl, e0);
  off(S.x_vmid, EN), off(S.x_cout, EN), off(S.x_vout, EN), off(S.x_deg, EN), off(S.x_isolv, IS);
  off(S.x_tab, e0 * tcap), off(S.x_adj, e0 * 2 * tcap), off(S.x_off, e0 * (N + 1)), off(S.x_dfs, e0 * tcap);
  off(S.spill_count, e0);
  off(S.sched, e0);  // a slice's order holds slice-local env ids (launch_env_order on the slice)
  if (B.sp_pool == 0) {  // one working-set slot per env: the slice's rows; a pool is shared as it is
    off(S.sp_tab, e0 * C), off(S.sp_adj, e0 * 2 * C), off(S.sp_ord, e0 * C), off(S.sp_cst, e0 * C);
    off(S.sp_cim, e0 * C), off(S.sp_lam, e0 * C);
    if (B.sp_rec) S.sp_rec = static_cast<float4*>(B.sp_rec) + EN * 3;  // 48-B records
  }
  return S;
}

// Step k's outputs: row k of [K, ...] buffers in the trajectory form (macm_world_rollout_traj),
// else the one set every step overwrites.
static macm_outputs step_outputs(const macm_world* w, const macm_outputs* out, int k, bool traj) {
  macm_outputs o = *out;
  if (!traj || k == 0) return o;
  const size_t E = w->P.n_envs, EN = E * w->P.n_agents;
  const size_t obytes = EN * obs_dim(w->cfg) * (w->cfg.obs_f64 ? sizeof(double) : sizeof(float));
  if (o.obs) o.obs = static_cast<unsigned char*>(o.obs) + k * obytes;
  if (o.nbr_id) o.nbr_id += k * EN;
  if (o.reward) o.reward += k * EN;
  if (o.collided) o.collided += k * EN;
  if (o.done) o.done += k * E;
  return o;
}

// Workgroup-path rollout over env slices on streams of their own. The step is three launches whose
// durations are each set by the slowest env, so the K steps of kSlices env slices run on their own
// streams with no join between steps: one slice's next kernels fill another's tails. Forked from
// and joined back into the caller's stream; results are those of the per-step launches (envs are
// independent). Measured at C3 (4096 x 256, steps 6-25): 568 -> 484 us per step with 2 slices,
// 481 with 3, but 744 with 4: with the caller's stream that is more streams than the process's 4
// hardware queues (GPU_MAX_HW_QUEUES), and two slices sharing a queue serialise each other's
// launches. C5 (N = 1024, 2048 envs) gained nothing (profiles/r02/rollout/).
static constexpr int kSlices = 3, kSliceMinEnvs = 1024, kSliceMaxAgents = 512;
// MACM_WG_SLICES=n: n env slices (0: none, the handoff instead; A/B sessions), kSlices by default
static int n_slices() {
  const char* v = getenv("MACM_WG_SLICES");
  const int n = v ? atoi(v) : kSlices;
  return n < 0 ? 0 : n > 8 ? 8 : n;
}
// the env slices a workgroup-path rollout of this world runs (0: none, one stream)
static int wg_rollout_slices(const macm_world* w) {
  if (w->wave || w->big || w->P.n_envs < kSliceMinEnvs || w->P.n_agents >= kSliceMaxAgents) return 0;
  const int S = n_slices();
  return S >= 2 ? S : 0;
}
// astride == 0: the closed loop (macm_world_rollout_bots): every step of a slice reads the bot's
// action rows of its envs and the bots kernel writes the next ones from the slice's obs rows
// (trajectory form: step k reads action row k and writes row k + 1 of [K + 1, E, N, 3]).
static int rollout_wg_slices(macm_world* w, int S, const unsigned char* actions, int n_steps,
                             unsigned long long astride, const macm_outputs* out, bool traj, hipStream_t user) {
  const int E = w->P.n_envs, N = w->P.n_agents;
  if ((int)w->slice_streams.size() < S) {
    for (int i = (int)w->slice_streams.size(); i < S; ++i) {
      hipStream_t st;
      HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      w->slice_streams.push_back(st);
    }
  }
  while ((int)w->slice_events.size() < S + 1) {
    hipEvent_t ev;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    w->slice_events.push_back(ev);
  }
  const size_t od = (size_t)N * obs_dim(w->cfg) * (w->cfg.obs_f64 ? sizeof(double) : sizeof(float));
  const bool bots = astride == 0;
  const size_t abytes = bots ? 3 * (size_t)N : astride / (size_t)E;
  const unsigned long long kstride = bots ? (traj ? (unsigned long long)E * abytes : 0ull) : astride;
  HIP_TRY(hipEventRecord(w->slice_events[0], user));
  std::vector<StepParams> Ps(S, w->P);
  std::vector<WorldBuffers> Bs(S);
  std::vector<size_t> e0s(S);
  for (int i = 0; i < S; ++i) {
    const size_t e0 = (size_t)E * i / S, e1 = (size_t)E * (i + 1) / S;
    e0s[i] = e0;
    Ps[i].n_envs = (int)(e1 - e0);
    Bs[i] = slice_buffers(w->B, e0, N, w->P.n_targets, w->P.max_contacts, w->tcap);
    HIP_TRY(hipStreamWaitEvent(w->slice_streams[i], w->slice_events[0], 0));
  }
  // every launch is enqueued before the join below; a failed launch still joins the slice streams
  // into the caller's (no unjoined work left behind) and leaves the list parity of
  // the steps that were launched
  int rc = MACM_OK, launched = 0;
  for (int k = 0; k < n_steps && rc == MACM_OK; ++k) {
    const int cur = w->cur ^ (k & 1);
    const macm_outputs ok = step_outputs(w, out, k, traj);
    for (int i = 0; i < S && rc == MACM_OK; ++i) {
      const size_t e0 = e0s[i];
      auto row = [e0](auto* p, size_t per_env) { return p ? p + e0 * per_env : p; };
      unsigned char* obs_i = ok.obs ? static_cast<unsigned char*>(ok.obs) + e0 * od : nullptr;
      const unsigned char* act_k = actions + k * kstride + e0 * abytes;
      // closed loop: kernel C takes the bot's next actions from the rows it writes (no bots launch)
      uint8_t* const bot = bots ? const_cast<unsigned char*>(act_k) + (traj ? (size_t)E * abytes : 0) : nullptr;
      const hipError_t he = launch_step_wg(Ps[i], Bs[i], cur, w->tcap, act_k, obs_i, w->cfg.obs_f64 != 0,
                                           row(ok.nbr_id, N), row(ok.reward, N), row(ok.collided, N),
                                           row(ok.done, 1), w->slice_streams[i], nullptr, bot);
      if (he != hipSuccess) rc = fail(MACM_E_HIP, std::string("rollout launch: ") + hipGetErrorString(he));
    }
    if (rc == MACM_OK) ++launched;
  }
  for (int i = 0; i < S; ++i) {
    HIP_TRY(hipEventRecord(w->slice_events[1 + i], w->slice_streams[i]));
    HIP_TRY(hipStreamWaitEvent(user, w->slice_events[1 + i], 0));
  }
  if (launched & 1) w->cur ^= 1;
  return rc;
}

// macm_world_rollout / _traj (bots = false) and macm_world_rollout_bots / _traj (bots = true)
static int world_rollout(macm_world* w, const void* actions, int n_steps, const macm_outputs* out, void* stream,
                         bool bots, bool traj) {
  if (n_steps < 0) return fail(MACM_E_INVALID, "n_steps must be >= 0");
  if (n_steps == 0) return MACM_OK;  // nothing is read, so actions may be NULL (an empty tensor)
  if (!w || !actions || !out || !out->reward) return fail(MACM_E_INVALID, "world/actions/out/reward is NULL");
  if (bots && !out->obs) return fail(MACM_E_INVALID, "out->obs is NULL (the bots act on it)");
  if (bots && w->cfg.action_mode != MACM_ACTION_DISCRETE) return fail(MACM_E_INVALID, "bots.flock acts in discrete mode");
  if (const uint32_t st = read_host_status(w->hstat)) return overflow_error(st);
  DeviceGuard g(w->device);
  hipStream_t s = (hipStream_t)stream;
  const int mode = w->cfg.action_mode == MACM_ACTION_DISCRETE ? 0 : 1;
  if (w->cfg.validate_actions) {  // every step's actions before any env is stepped (bots: the caller's first)
    const long long rows = (long long)(bots ? 1 : n_steps) * w->P.n_envs;
    if (rows > INT32_MAX) return fail(MACM_E_INVALID, "n_steps * n_envs too large to validate");
    const int rc = check_actions(w->bad, actions, mode, nullptr, (int)rows, w->P.n_agents, s, w->P.n_envs);
    if (rc) return rc;
  }
  const unsigned long long astride =
      bots ? 0ull
           : (unsigned long long)w->P.n_envs * w->P.n_agents * (mode == 0 ? 3 * sizeof(uint8_t) : 2 * sizeof(float));
  if (w->wave) {  // one launch; astride 0: the closed-loop form of the rollout kernel
    HIP_TRY(launch_rollout_w64(w->P, w->B, w->cur, actions, out->obs, w->cfg.obs_f64 != 0, out->nbr_id, out->reward,
                               out->collided, out->done, s, n_steps, astride, traj ? 1 : 0));
    if (n_steps & 1) w->cur ^= 1;
    return MACM_OK;
  }
  const unsigned char* act = static_cast<const unsigned char*>(actions);
  if (const int S = wg_rollout_slices(w)) return rollout_wg_slices(w, S, act, n_steps, astride, out, traj, s);
  // workgroup path: its three launches per step (and the bot's), in order
  const long long rows = (long long)w->P.n_envs * w->P.n_agents;
  const unsigned long long kstride = bots ? (traj ? (unsigned long long)rows * 3 : 0ull) : astride;
  for (int k = 0; k < n_steps; ++k) {
    const macm_outputs ok = step_outputs(w, out, k, traj);
    const unsigned char* act_k = act + k * kstride;
    if (w->big)
      HIP_TRY(launch_step_big(w->P, w->B, w->cur, act_k, ok.obs, w->cfg.obs_f64 != 0, ok.nbr_id, ok.reward,
                              ok.collided, ok.done, s));
    else
      HIP_TRY(launch_step_wg(w->P, w->B, w->cur, w->tcap, act_k, ok.obs, w->cfg.obs_f64 != 0, ok.nbr_id, ok.reward,
                             ok.collided, ok.done, s, handoff_for(w),
                             bots ? const_cast<unsigned char*>(act_k) + (traj ? rows * 3 : 0) : nullptr));
    w->cur ^= 1;
    if (bots && w->big)
      HIP_TRY(launch_bots_flock(ok.obs, w->cfg.obs_f64 != 0, obs_dim(w->cfg), rows,
                                const_cast<unsigned char*>(act_k) + (traj ? rows * 3 : 0), s));
  }
  return MACM_OK;
}

int macm_world_rollout(macm_world* w, const void* actions, int n_steps, const macm_outputs* out, void* stream) {
  return world_rollout(w, actions, n_steps, out, stream, false, false);
}

int macm_world_rollout_traj(macm_world* w, const void* actions, int n_steps, const macm_outputs* traj,
                            void* stream) {
  return world_rollout(w, actions, n_steps, traj, stream, false, true);
}

int macm_world_rollout_bots(macm_world* w, uint8_t* actions, int n_steps, const macm_outputs* out, void* stream) {
  return world_rollout(w, actions, n_steps, out, stream, true, false);
}

int macm_world_rollout_bots_traj(macm_world* w, uint8_t* actions, int n_steps, const macm_outputs* traj,
                                 void* stream) {
  return world_rollout(w, actions, n_steps, traj, stream, true, true);
}

int macm_world_observe(macm_world* w, const macm_outputs* out, void* stream) {
  if (!w || !out) return fail(MACM_E_INVALID, "world/out is NULL");
  DeviceGuard g(w->device);
  if (w->wave)
    HIP_TRY(launch_observe_w64(w->P, w->B, out->obs, w->cfg.obs_f64 != 0, out->nbr_id, (hipStream_t)stream));
  else if (w->big)
    HIP_TRY(launch_observe_big(w->P, w->B, out->obs, w->cfg.obs_f64 != 0, out->nbr_id, (hipStream_t)stream));
  else
    HIP_TRY(launch_observe_wg(w->P, w->B, out->obs, w->cfg.obs_f64 != 0, out->nbr_id, (hipStream_t)stream));
  return MACM_OK;
}

// Rows of E contact lists between the caller's [E, stride] layout and the world's [E, C] buffers:
// the first min(stride, C) entries of each row (the rest of a device row is never read, the rest
// of a caller's row is left as it is).
static hipError_t copy_rows(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t E,
                            hipStream_t s) {
  if (E == 0 || width == 0) return hipSuccess;
  return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, E, hipMemcpyDefault, s);
}

// set_state's contact lists: staged in the spare list buffer (cur ^ 1: the next step's output, unused
// between steps) and validated there on the device (a host loop over E x C entries).
// On success the caller flips its `cur` to take them; on failure nothing of the world changed.
static int stage_lists(WorldBuffers& B, int cur, unsigned long long* bad, size_t E, size_t C, size_t Cs, int N,
                       const void* count, const void* ab, const void* imp, hipStream_t s) {
  const int nb = cur ^ 1;
  const size_t Cw = Cs < C ? Cs : C;
  HIP_TRY(hipMemcpyAsync(B.ccount[nb], count, E * sizeof(int32_t), hipMemcpyDefault, s));
  HIP_TRY(copy_rows(B.cab[nb], C * sizeof(uint32_t), ab, Cs * sizeof(uint32_t), Cw * sizeof(uint32_t), E, s));
  HIP_TRY(hipMemsetAsync(bad, 0xff, sizeof(unsigned long long), s));
  HIP_TRY(launch_check_lists(B.ccount[nb], B.cab[nb], (int)E, (int)C, (int)Cw, N, bad, s));
  unsigned long long h = ~0ull;
  HIP_TRY(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (h != ~0ull) {
    const unsigned long long e = h >> 32, k = h & 0xffffffffull;
    if (k == 0xffffffffull)
      return fail(MACM_E_INVALID, "env " + std::to_string(e) + ": contact_count outside [0, min(max_contacts = " +
                                      std::to_string(C) + ", contact_stride = " + std::to_string(Cs) + ")]");
    return fail(MACM_E_INVALID, "env " + std::to_string(e) + ": contact_ab[" + std::to_string(k) +
                                    "] is not a pair a < b < n_agents");
  }
  if (imp)
    HIP_TRY(copy_rows(B.cimp[nb], C * sizeof(float2), imp, Cs * sizeof(float2), Cw * sizeof(float2), E, s));
  else
    HIP_TRY(hipMemsetAsync(B.cimp[nb], 0, E * C * sizeof(float2), s));
  return MACM_OK;
}

static int copy_state(macm_world* w, const macm_state* st, void* stream, bool to_device) {
  if (!w || !st) return fail(MACM_E_INVALID, "world/state is NULL");
  if (st->contact_stride < 0) return fail(MACM_E_INVALID, "contact_stride must be >= 0");
  DeviceGuard g(w->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t E = w->P.n_envs, N = w->P.n_agents, T = w->P.n_targets, C = w->P.max_contacts;
  const size_t Cs = st->contact_stride > 0 ? (size_t)st->contact_stride : C;  // the caller's row length
  const size_t Cw = Cs < C ? Cs : C;                                           // entries moved per row
  if (to_device) {
    if (!st->contact_count != !st->contact_ab)
      return fail(MACM_E_INVALID, "contact_count and contact_ab must be given together");
    if (st->contact_count) {
      const int rc = stage_lists(w->B, w->cur, w->bad, E, C, Cs, (int)N, st->contact_count, st->contact_ab,
                                 st->contact_imp, s);
      if (rc) return rc;
      w->cur ^= 1;
    }
    HIP_TRY(hipStreamSynchronize(s));
    clear_host_status(w->hstat);  // an injected state starts clean
    HIP_TRY(hipMemsetAsync(w->B.status, 0, E * sizeof(int32_t), s));
  } else {
    if (st->contact_count)
      HIP_TRY(hipMemcpyAsync(st->contact_count, w->B.ccount[w->cur], E * sizeof(int32_t), hipMemcpyDefault, s));
    if (st->contact_ab)
      HIP_TRY(copy_rows(st->contact_ab, Cs * sizeof(uint32_t), w->B.cab[w->cur], C * sizeof(uint32_t),
                        Cw * sizeof(uint32_t), E, s));
    if (st->contact_imp)
      HIP_TRY(copy_rows(st->contact_imp, Cs * sizeof(float2), w->B.cimp[w->cur], C * sizeof(float2),
                        Cw * sizeof(float2), E, s));
  }
  struct Item {
    void* user;
    void* dev;
    size_t bytes;
  } items[] = {
      {st->pos, w->B.pos, E * N * sizeof(float2)},
      {st->vel, w->B.vel, E * N * sizeof(float2)},
      {st->angle, w->B.angle, E * N * sizeof(float)},
      {st->fat, w->B.fat, E * N * sizeof(float4)},
      {st->sleep, w->B.sleep, E * N * sizeof(float)},
      {st->targets, w->B.targets, E * T * sizeof(float2)},
      {st->step_count, w->B.step_count, E * sizeof(int32_t)},
      {st->time_passed, w->B.time_passed, E * sizeof(double)},
  };
  for (const Item& it : items) {
    if (!it.user) continue;
    if (to_device) HIP_TRY(hipMemcpyAsync(it.dev, it.user, it.bytes, hipMemcpyDefault, s));
    else HIP_TRY(hipMemcpyAsync(it.user, it.dev, it.bytes, hipMemcpyDefault, s));
  }
  if (to_device && st->time_passed) {
    // done flag follows time_passed (mvmnt.py:135-136)
    std::vector<double> tp(E);
    std::vector<uint8_t> dn(E);
    HIP_TRY(hipMemcpyAsync(tp.data(), w->B.time_passed, E * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (size_t e = 0; e < E; ++e) dn[e] = tp[e] > w->P.time_limit ? 1 : 0;
    HIP_TRY(hipMemcpyAsync(w->B.done, dn.data(), E, hipMemcpyHostToDevice, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return MACM_OK;
}

int macm_world_get_state(macm_world* w, const macm_state* dst, void* stream) {
  return copy_state(w, dst, stream, false);
}

int macm_world_set_state(macm_world* w, const macm_state* src, void* stream) {
  return copy_state(w, src, stream, true);
}

int macm_world_status(macm_world* w, int32_t* status_or, void* stream) {
  if (!w || !status_or) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  std::vector<int32_t> st(w->P.n_envs);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(st.data(), w->B.status, st.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  int32_t acc = 0;
  for (int32_t v : st) acc |= v;
  *status_or = acc;
  return MACM_OK;
}

int macm_world_counters(macm_world* w, int64_t out[4], void* stream) {
  if (!w || !out) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  std::vector<unsigned long long> h((size_t)w->P.n_envs * 4);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(h.data(), w->B.env_counters, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                         s));
  HIP_TRY(hipStreamSynchronize(s));
  unsigned long long acc[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < h.size(); ++i) acc[i & 3] += h[i];
  for (int i = 0; i < 4; ++i) out[i] = (int64_t)acc[i];
  return MACM_OK;
}

int macm_world_reset_counters(macm_world* w, void* stream) {
  if (!w) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  HIP_TRY(hipMemsetAsync(w->B.env_counters, 0, (size_t)w->P.n_envs * 4 * sizeof(unsigned long long),
                         (hipStream_t)stream));
  HIP_TRY(hipMemsetAsync(w->B.env_rsum, 0, (size_t)w->P.n_envs * sizeof(double), (hipStream_t)stream));
  return MACM_OK;
}

// Per-env reward sums (flock_common.hpp: each step's float32 rewards as float64, pairwise over the
// agent slots, added to the env's total in step order) and their sum over envs in env order, starting
// from +0.0: a fixed order throughout, so the total is bit-stable for any launch form or env slicing.
// Binary rewards are -1, 0 or +1, so every partial sum in that order is an exact integer and an env's
// total is exactly (positive-reward agent-steps) - (collided agent-steps), its counters 2 and 1: the
// kernels accumulate env_rsum for linear rewards only (a binary world's per-step sum and atomic add
// cost 2.5% of the steady-state step, profiles/r06/abtests/rsum/).
int macm_world_reward_sums(macm_world* w, double* per_env, double* total, void* stream) {
  if (!w || (!per_env && !total)) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  std::vector<double> h((size_t)w->P.n_envs);
  hipStream_t s = (hipStream_t)stream;
  if (w->P.reward_mode == MACM_REWARD_LINEAR) {
    HIP_TRY(hipMemcpyAsync(h.data(), w->B.env_rsum, h.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  } else {
    std::vector<unsigned long long> c(h.size() * 4);
    HIP_TRY(hipMemcpyAsync(c.data(), w->B.env_counters, c.size() * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (size_t e = 0; e < h.size(); ++e) h[e] = (double)((long long)c[e * 4 + 2] - (long long)c[e * 4 + 1]);
  }
  if (per_env) memcpy(per_env, h.data(), h.size() * sizeof(double));
  if (total) {
    double acc = 0.0;
    for (double v : h) acc += v;
    *total = acc;
  }
  return MACM_OK;
}

int macm_world_spilled(macm_world* w, int64_t* env_steps, void* stream) {
  if (!w || !env_steps) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  std::vector<uint32_t> h((size_t)w->P.n_envs);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(h.data(), w->B.spill_count, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  int64_t acc = 0;
  for (uint32_t v : h) acc += v;
  *env_steps = acc;
  return MACM_OK;
}

// MACM_DEBUG_SPILL_POOL (a test hook): share `pool` of the slots allocated at creation;
// MACM_DEBUG_SPILL_FAIL: no slot is ever free (every spilling env ends SPILL_WAIT); a call
// without either flag brings back the world's own pool (or one slot per env). The locks are cleared
// only after the device has finished every step that could hold one.
extern "C++" template <typename Wt>
static int set_spill_pool(Wt* w, int32_t flags, int pool) {
  const bool want = (flags & MACM_DEBUG_SPILL_POOL) != 0;
  const bool never = (flags & MACM_DEBUG_SPILL_FAIL) != 0;
  if (want && never) return fail(MACM_E_INVALID, "SPILL_POOL and SPILL_FAIL exclude each other");
  if (want && (pool < 1 || pool > w->slots_alloc))
    return fail(MACM_E_INVALID, "SPILL_POOL: 1 <= slots <= the " + std::to_string(w->slots_alloc) + " allocated");
  const int target = never ? -1 : want ? pool : w->pool0;  // -1: acquire_slot always fails
  if (target == w->B.sp_pool) return MACM_OK;
  DeviceGuard g(w->device);
  HIP_TRY(hipDeviceSynchronize());
  if (target > 0) {
    if (!w->B.sp_lock && dalloc(w->allocs, &w->B.sp_lock, (size_t)w->slots_alloc)) return MACM_E_OOM;
    HIP_TRY(hipMemset(w->B.sp_lock, 0, sizeof(uint32_t) * w->slots_alloc));
  }
  w->B.sp_pool = target;
  return MACM_OK;
}

int macm_world_set_debug(macm_world* w, int32_t flags) {
  if (!w) return fail(MACM_E_INVALID, "world is NULL");
  const int pool = (flags & MACM_DEBUG_SPILL_POOL) ? (flags >> 8) : 0;
  flags &= 0xff;
  if (flags & ~(MACM_DEBUG_FORCE_SPILL | MACM_DEBUG_SWEEP_CELLS | MACM_DEBUG_SWEEP_ALL_PAIRS | MACM_DEBUG_SPILL_POOL | MACM_DEBUG_SPILL_FAIL))
    return fail(MACM_E_INVALID, "unknown debug flag");
  if ((flags & MACM_DEBUG_SWEEP_CELLS) && (flags & MACM_DEBUG_SWEEP_ALL_PAIRS))
    return fail(MACM_E_INVALID, "SWEEP_CELLS and SWEEP_ALL_PAIRS exclude each other");
  if (int rc = set_spill_pool(w, flags, pool)) return rc;
  w->P.force_spill = (flags & MACM_DEBUG_FORCE_SPILL) ? 1 : 0;
  w->P.sweep = (flags & MACM_DEBUG_SWEEP_CELLS) ? 1 : (flags & MACM_DEBUG_SWEEP_ALL_PAIRS) ? 2 : 0;
  return MACM_OK;
}

// ============================ TDM =============================================

int macm_tdm_config_default(macm_tdm_config* c) {
  if (!c) return fail(MACM_E_INVALID, "cfg is NULL");
  memset(c, 0, sizeof(*c));
  c->n_teams = 2;  // TDM(n_agents=[1, 1]) default, combat.py:62
  c->team_size[0] = 1;
  c->team_size[1] = 1;
  c->n_agents = 2;
  c->velocity_iterations = 8;
  c->position_iterations = 3;
  c->warm_starting = 1;
  c->obs_f64 = 0;
  c->fresh_raycast = 0;
  c->decay_mov_penalty = 0;
  c->hz = 60.0;
  c->world_width = 30.0;
  c->world_height = 30.0;
  c->agent_rotation_speed = 0.8 * (2 * M_PI);
  c->agent_force = 20.0;
  c->percent_mov_penalty = 0.2;
  c->melee_range = 2.0;
  c->melee_dmg = 0.25;
  c->init_health = 1.0;
  c->cooldown_atk = 1.0;
  c->cooldown_mov_penalty = 0.5;
  c->time_limit = 60.0;
  c->radius = 0.5f;
  c->density = 1.0f;
  c->friction = 0.3f;
  c->linear_damping = 5.0f;
  return MACM_OK;
}

static void free_tdm(macm_tdm* w) {
  for (void* p : w->allocs) (void)hipFree(p);
  w->allocs.clear();
  if (w->snap) (void)hipFree(w->snap);
  w->snap = nullptr;
  if (w->tail_snap) (void)hipFree(w->tail_snap);
  w->tail_snap = nullptr;
  if (w->tail_ctl) (void)hipFree(w->tail_ctl);
  w->tail_ctl = nullptr;
  if (w->obs_stream) (void)hipStreamDestroy(w->obs_stream);
  w->obs_stream = nullptr;
  for (int b = 0; b < 2; ++b) {
    if (w->ev_phys[b]) (void)hipEventDestroy(w->ev_phys[b]);
    if (w->ev_obs[b]) (void)hipEventDestroy(w->ev_obs[b]);
    w->ev_phys[b] = w->ev_obs[b] = nullptr;
  }
  if (w->hstat) (void)hipHostFree(w->hstat);
  w->hstat = nullptr;
}

int macm_tdm_create(const macm_tdm_config* cfg, int32_t n_envs, int32_t device, macm_tdm** out) {
  if (!cfg || !out) return fail(MACM_E_INVALID, "cfg/out is NULL");
  *out = nullptr;
  const macm_tdm_config& c = *cfg;
  if (n_envs <= 0) return fail(MACM_E_INVALID, "n_envs must be > 0");
  if (c.n_teams < 1 || c.n_teams > 4) return fail(MACM_E_INVALID, "n_teams must be in [1, 4]");
  int N = 0;
  for (int t = 0; t < c.n_teams; ++t) {
    if (c.team_size[t] < 0) return fail(MACM_E_INVALID, "team_size < 0");
    N += c.team_size[t];
  }
  if (N != c.n_agents) return fail(MACM_E_INVALID, "n_agents != sum(team_size)");
  if (N < 2) return fail(MACM_E_INVALID, "n_agents must be >= 2");
  // N > 64: the workgroup step (tdm_step_wg.hip), one thread per agent and 16-bit body ids in the
  // contact list, as the Flock workgroup path
  if (N > kMaxAgents) return fail(MACM_E_UNSUPPORTED, "TDM with more than 4096 agents per env is not built");
  if (!(c.hz > 0.0)) return fail(MACM_E_INVALID, "hz must be > 0");
  if (c.velocity_iterations < 0 || c.position_iterations < 0) return fail(MACM_E_INVALID, "iterations < 0");
  if (!(c.radius > 0.0f)) return fail(MACM_E_INVALID, "radius must be > 0");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MACM_E_INVALID, "device index out of range");
  DeviceGuard g(device);
  size_t free_bytes = 0, total_bytes = 0;
  HIP_TRY(hipMemGetInfo(&free_bytes, &total_bytes));
  if (N > 64) {
    int max_lds = 0;
    HIP_TRY(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device));
    const int need = std::max(tdm_wg_step_lds(N), tdm_wg_obs_lds(N));
    if (need > max_lds)
      return fail(MACM_E_UNSUPPORTED, "TDM workgroup step needs " + std::to_string(need) + " B of LDS, device has " +
                                          std::to_string(max_lds));
    HIP_TRY(tdm_wg_configure(N));
  }

  macm_tdm* w = new macm_tdm();
  w->cfg = c;
  w->device = device;
  w->cur = 0;
  w->wave = N <= 64;
  const int C = N * (N - 1) / 2;  // every pair: the list never overflows
  // spill working-set slots from the device budget, as Flock's: one per env when they fit, else a
  // pool. Both TDM callers take their slot before committing anything of the step (the wave
  // kernel's hand-over and the workgroup step), so a pool wait leaves an env wholly unstepped,
  // never half-stepped (N <= 64 used to take one slot per env regardless of memory)
  const int64_t SL = default_capacity(N, n_envs, C, free_bytes).slots;
  StepParams& P = w->P;
  memset(&P, 0, sizeof(P));
  P.n_envs = n_envs;
  P.n_agents = N;
  P.n_targets = 0;
  P.max_contacts = C;
  P.vel_iters = c.velocity_iterations;
  P.pos_iters = c.position_iterations;
  P.warm_starting = c.warm_starting ? 1 : 0;
  P.action_mode = MACM_ACTION_DISCRETE;
  P.reward_mode = MACM_REWARD_BINARY;
  P.coord = MACM_COORD_POLAR;
  fill_body_params(P, c.hz, c.radius, c.density, c.friction, c.linear_damping, c.agent_force,
                   c.agent_rotation_speed);
  P.time_limit = c.time_limit;
  TdmParams& TP = w->TP;
  memset(&TP, 0, sizeof(TP));
  TP.n_teams = c.n_teams;
  for (int t = 0, acc = 0; t < 4; ++t) {
    acc += t < c.n_teams ? c.team_size[t] : 0;
    TP.team_end[t] = acc;
  }
  TP.fresh_raycast = c.fresh_raycast ? 1 : 0;
  TP.decay_mov_penalty = c.decay_mov_penalty ? 1 : 0;
  TP.melee_range = c.melee_range;
  TP.melee_dmg = c.melee_dmg;
  TP.cooldown_atk = c.cooldown_atk;
  TP.cooldown_mov_penalty = c.cooldown_mov_penalty;
  TP.percent_mov_penalty = c.percent_mov_penalty;
  TP.init_health = c.init_health;
  w->team.resize(N);
  for (int i = 0; i < N; ++i) w->team[i] = tdm_team_of(TP, i);

  WorldBuffers& B = w->B;
  TdmBuffers& TB = w->TB;
  memset(&B, 0, sizeof(B));
  memset(&TB, 0, sizeof(TB));
  const size_t EN = (size_t)n_envs * N, E = (size_t)n_envs;
  std::vector<void*>& A = w->allocs;
  int rc = MACM_OK;
  if ((rc = dalloc(A, &B.pos, EN)) || (rc = dalloc(A, &B.vel, EN)) || (rc = dalloc(A, &B.angle, EN)) ||
      (rc = dalloc(A, &B.fat, EN)) || (rc = dalloc(A, &B.sleep, EN)) || (rc = dalloc(A, &B.ccount[0], E)) ||
      (rc = dalloc(A, &B.ccount[1], E)) || (rc = dalloc(A, &B.cab[0], E * C)) ||
      (rc = dalloc(A, &B.cab[1], E * C)) || (rc = dalloc(A, &B.cimp[0], E * C)) ||
      (rc = dalloc(A, &B.cimp[1], E * C)) || (rc = dalloc(A, &B.step_count, E)) ||
      (rc = dalloc(A, &B.time_passed, E)) || (rc = dalloc(A, &B.done, E)) || (rc = dalloc(A, &B.status, E)) ||
      (rc = dalloc(A, &B.env_counters, E * 4)) || (rc = dalloc(A, &TB.health, EN)) ||
      (rc = dalloc(A, &TB.cd_atk, EN)) || (rc = dalloc(A, &TB.cd_mov, EN)) || (rc = dalloc(A, &TB.alive, EN)) ||
      (rc = dalloc(A, &TB.listener, E)) || (rc = dalloc(A, &TB.winner, E)) || (rc = dalloc(A, &w->bad, 1)) ||
      (rc = dalloc(A, &w->mt, E * kMtStride)) || (rc = dalloc(A, &w->rmask, E)) ||
      // the spill step's working set (an env with more than 256 touching contacts or 16 per body):
      // C = every pair; its body records in HBM too (the TDM kernel's LDS pool holds the rest)
      (rc = dalloc(A, &B.sp_tab, (size_t)SL * C)) || (rc = dalloc(A, &B.sp_adj, (size_t)SL * 2 * C)) ||
      (rc = dalloc(A, &B.sp_ord, (size_t)SL * C)) || (rc = dalloc(A, &B.sp_cst, (size_t)SL * C)) ||
      (rc = dalloc(A, &B.sp_cim, (size_t)SL * C)) || (rc = dalloc(A, &B.sp_lam, (size_t)SL * C)) ||
      (rc = dalloc(A, (float4**)&B.sp_rec, (size_t)SL * N * 3)) ||  // 48-B records
      (SL < n_envs && (rc = dalloc(A, &B.sp_lock, (size_t)SL))) || (rc = dalloc(A, &B.spill_count, E)) ||
      (w->wave && (rc = dalloc(A, &B.sched, (size_t)E)))
#ifdef MACM_STAMPS
      || (rc = dalloc(A, &B.stamps, E * 32))
#endif
  ) {
    free_tdm(w);
    delete w;
    return rc;
  }
  if (hipError_t he = alloc_host_status(&w->hstat, &B.host_status); he != hipSuccess) {
    free_tdm(w);
    delete w;
    return fail(MACM_E_OOM, std::string("hipHostMalloc (status word): ") + hipGetErrorString(he));
  }
  hipError_t e = hipMemset(B.env_counters, 0, E * 4 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(B.ccount[0], 0, sizeof(int32_t) * E);
  if (e == hipSuccess) e = hipMemset(B.status, 0, sizeof(int32_t) * E);
  if (e == hipSuccess) e = hipMemset(B.spill_count, 0, sizeof(uint32_t) * E);
  B.sp_pool = SL < n_envs ? (int32_t)SL : 0;
  w->slots_alloc = (int)SL;
  w->pool0 = B.sp_pool;
  if (e == hipSuccess && B.sp_lock) e = hipMemset(B.sp_lock, 0, sizeof(uint32_t) * SL);
  if (e != hipSuccess) {
    free_tdm(w);
    delete w;
    return fail(MACM_E_HIP, std::string("tdm init: ") + hipGetErrorString(e));
  }
  *out = w;
  return MACM_OK;
}

int macm_tdm_destroy(macm_tdm* w) {
  if (!w) return MACM_OK;
  DeviceGuard g(w->device);
  (void)hipDeviceSynchronize();
  free_tdm(w);
  delete w;
  return MACM_OK;
}

static TdmBuffers tdm_with_outputs(const macm_tdm* w, const macm_tdm_outputs* out) {
  TdmBuffers TB = w->TB;
  if (out) {
    TB.mask_out = out->mask;
    TB.health_out = out->health;
    TB.alive_out = out->alive;
    TB.winner_out = out->winner;
  }
  return TB;
}

static hipError_t tdm_launch_init(const macm_tdm* w, const TdmBuffers& TB, void* obs, const uint8_t* mask,
                                  hipStream_t s) {
  if (w->wave) return launch_tdm_init_w64(w->P, w->B, w->TP, TB, w->cur, obs, w->cfg.obs_f64 != 0, mask, s);
  return launch_tdm_init_wg(w->P, w->B, w->TP, TB, w->cur, obs, w->cfg.obs_f64 != 0, mask, s);
}

static hipError_t tdm_launch_step(const macm_tdm* w, const TdmBuffers& TB, int cur, const void* actions, void* obs,
                                  uint8_t* done, hipStream_t s) {
  if (w->wave) return launch_tdm_step_w64(w->P, w->B, w->TP, TB, cur, actions, obs, w->cfg.obs_f64 != 0, done, s);
  return launch_tdm_step_wg(w->P, w->B, w->TP, TB, cur, actions, obs, w->cfg.obs_f64 != 0, done, s);
}

static int tdm_init(macm_tdm* w, const macm_tdm_outputs* out, hipStream_t s) {
  HIP_TRY(hipStreamSynchronize(s));  // earlier steps' status stores land before the word is cleared
  clear_host_status(w->hstat);
  w->cur = 0;
  const TdmBuffers TB = tdm_with_outputs(w, out);
  HIP_TRY(tdm_launch_init(w, TB, out ? out->obs : nullptr, nullptr, s));
  if (out && out->done) HIP_TRY(hipMemsetAsync(out->done, 0, (size_t)w->P.n_envs, s));
  return MACM_OK;
}

int macm_tdm_reset(macm_tdm* w, uint64_t seed, int64_t env_offset, const macm_tdm_outputs* out, void* stream) {
  if (!w) return fail(MACM_E_INVALID, "tdm is NULL");
  DeviceGuard g(w->device);
  const macm_tdm_config& c = w->cfg;
  const int E = w->P.n_envs, N = w->P.n_agents;
  std::vector<float2> pos((size_t)E * N);
  std::vector<float> ang((size_t)E * N);
  std::vector<uint32_t> mts((size_t)E * kMtStride);
  for (int e = 0; e < E; ++e) {
    PyMT19937 r(seed + (uint64_t)(env_offset + e));
    for (int i = 0; i < N; ++i) {  // combat.py:80-95
      const double x = r.random() * (w->team[i] + c.world_width / 2);
      const double y = r.random() * c.world_height;
      const double a = r.uniform(-1, 1) * M_PI;
      pos[(size_t)e * N + i] = make_float2((float)x, (float)y);
      ang[(size_t)e * N + i] = (float)a;
    }
    save_stream(mts, e, r);
  }
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(w->B.pos, pos.data(), pos.size() * sizeof(float2), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(w->B.angle, ang.data(), ang.size() * sizeof(float), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(w->mt, mts.data(), mts.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  w->mt_valid = true;
  int rc = tdm_init(w, out, s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s));  // host vectors feed the async copies
  return MACM_OK;
}

int macm_tdm_place(macm_tdm* w, const void* pos, const void* angle, const macm_tdm_outputs* out, void* stream) {
  if (!w || !pos || !angle) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  const size_t EN = (size_t)w->P.n_envs * w->P.n_agents;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(w->B.pos, pos, EN * sizeof(float2), hipMemcpyDefault, s));
  HIP_TRY(hipMemcpyAsync(w->B.angle, angle, EN * sizeof(float), hipMemcpyDefault, s));
  w->mt_valid = false;  // poses came from the caller's generator
  int rc = tdm_init(w, out, s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return MACM_OK;
}

int macm_tdm_reset_envs(macm_tdm* w, const uint8_t* env_mask, const macm_tdm_outputs* out, void* stream) {
  if (!w) return fail(MACM_E_INVALID, "tdm is NULL");
  if (!w->mt_valid)
    return fail(MACM_E_INVALID, "no per-env random streams: the world was placed, not reset (macm_tdm_reset)");
  DeviceGuard g(w->device);
  hipStream_t s = (hipStream_t)stream;
  int rc = fill_reset_mask(w->rmask, env_mask, w->P.n_envs, s);
  if (rc) return rc;
  PoseDraw D;
  memset(&D, 0, sizeof(D));
  D.mode = kTdm;
  D.n_agents = w->P.n_agents;
  D.half_width = w->cfg.world_width / 2;
  D.height = w->cfg.world_height;
  D.TP = w->TP;
  HIP_TRY(launch_draw_poses(w->rmask, w->mt, D, w->P.n_envs, w->B.pos, w->B.angle, s));
  const TdmBuffers TB = tdm_with_outputs(w, out);
  HIP_TRY(tdm_launch_init(w, TB, out ? out->obs : nullptr, w->rmask, s));
  return resync_host_status(w->hstat, w->B.status, w->P.n_envs, s);
}

// The split observation (round 6, tdm_obs_snap.hip). The wave kernel (N <= 64) observes on its one
// wave after the physics: 55% of its cycles at 2 x 16 (tools/tdm_phase.py). With fewer envs than
// SIMDs (BASELINE C4's per-GPU shard: 512 envs, 0.5 waves per SIMD) that observation is one wave's
// latency chain. Split, the step writes pose snapshots and tdm_observe_snap observes every
// (step, env) row with a workgroup of its own; a trajectory rollout runs in chunks of
// kTdmSplitChunk steps, each chunk's observation on a second stream beside the next chunk's physics.
// Bit-identical either way. Measured (profiles/r06/split/, 2 x 16, one box): 512 envs 13.2 -> 11.6 us
// per step at steady state, 18.8 -> 18.1 us in the driver's window; 1024 envs even; 2048 and 4096 envs
// slower (26 / 50 us against 20 / 28: with every SIMD busy the observation kernel only competes with
// the physics). The physics alone takes ~11 us per step at 512 envs (rocprof: the chunk launches),
// one wave's latency chain, which bounds the shard whatever the observation costs.
// Below kTdmSplitMaxEnvs envs by default; MACM_TDM_SPLIT_OBS=0/1 overrides
// (tests, A/B). The closed loop (the bots read each step's observation inside the launch) and the
// workgroup step (N > 64) keep the fused form.
static constexpr int kTdmSplitMaxEnvs = 1024, kTdmSplitChunk = 8;

static bool tdm_split_obs(const macm_tdm* w) {
  if (!w->wave) return false;
  const char* v = getenv("MACM_TDM_SPLIT_OBS");
  return v ? atoi(v) != 0 : w->P.n_envs < kTdmSplitMaxEnvs;
}

// snapshot halves of at least `rows` rows each (grown on demand; the caller's stream has finished
// every earlier use: each split call ends with the stream joined to the observation stream)
static int tdm_split_buffers(macm_tdm* w, size_t rows, hipStream_t s) {
  if (!w->obs_stream) {
    HIP_TRY(hipStreamCreateWithFlags(&w->obs_stream, hipStreamNonBlocking));
    for (int b = 0; b < 2; ++b) {
      HIP_TRY(hipEventCreateWithFlags(&w->ev_phys[b], hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&w->ev_obs[b], hipEventDisableTiming));
    }
  }
  if (rows > w->snap_rows) {
    // at least a whole chunk's rows at the first allocation (a warm-up rollout shorter than a chunk
    // would otherwise leave the next rollout a synchronising reallocation)
    const size_t chunk = (size_t)kTdmSplitChunk * w->P.n_envs;
    if (rows < chunk) rows = chunk;
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipStreamSynchronize(w->obs_stream));
    if (w->snap) HIP_TRY(hipFree(w->snap));
    w->snap = nullptr;
    w->snap_rows = 0;
    if (hipMalloc(&w->snap, 2 * rows * (size_t)w->P.n_agents * sizeof(float4)) != hipSuccess) {
      (void)hipGetLastError();
      w->snap = nullptr;
      return fail(MACM_E_OOM, "hipMalloc (split observation snapshots)");
    }
    w->snap_rows = rows;
  }
  return MACM_OK;
}

int macm_tdm_step(macm_tdm* w, const void* actions, const macm_tdm_outputs* out, void* stream) {
  if (!w || !actions) return fail(MACM_E_INVALID, "tdm/actions is NULL");
  if (const uint32_t st = read_host_status(w->hstat)) return overflow_error(st);
  DeviceGuard g(w->device);
  if (w->cfg.validate_actions) {
    const int rc = check_actions(w->bad, actions, 2, w->TB.alive, w->P.n_envs, w->P.n_agents, (hipStream_t)stream);
    if (rc) return rc;
  }
  TdmBuffers TB = tdm_with_outputs(w, out);
  hipStream_t s = (hipStream_t)stream;
  void* obs = out ? out->obs : nullptr;
  if ((obs || TB.mask_out) && tdm_split_obs(w)) {
    const int rc = tdm_split_buffers(w, (size_t)w->P.n_envs, s);
    if (rc) return rc;
    TB.snap_out = w->snap;
    HIP_TRY(tdm_launch_step(w, TB, w->cur, actions, nullptr, out->done, s));
    w->cur ^= 1;
    HIP_TRY(launch_tdm_observe_snap(w->TP, w->P.n_agents, (size_t)w->P.n_envs, w->snap, obs, w->cfg.obs_f64 != 0,
                                    TB.mask_out, s));
    return MACM_OK;
  }
  HIP_TRY(tdm_launch_step(w, TB, w->cur, actions, obs, out ? out->done : nullptr, s));
  w->cur ^= 1;
  return MACM_OK;
}

// The tail observation (flock_step_w64.hip TailObs): a trajectory rollout of the wave kernel whose
// launch is wholly resident (the envs plus the observe-only blocks within the kernel's occupancy on
// this device). MACM_TDM_TAIL_OBS=0/1 overrides the default; MACM_TDM_TAIL_WORKERS sets the number
// of observe-only blocks (default: as many as the envs, within the resident capacity).
static int tdm_tail_workers(macm_tdm* w) {
  if (!w->wave) return -1;
  if (w->tail_cap < 0) w->tail_cap = tdm_rollout_resident_blocks(w->P.n_agents, w->cfg.obs_f64 != 0);
  const int E = w->P.n_envs, room = w->tail_cap - E;
  if (room < 0) return -1;
  const char* v = getenv("MACM_TDM_TAIL_WORKERS");
  int x = v ? atoi(v) : E;
  if (x < 0) x = 0;
  return x < room ? x : room;
}

// measured (profiles/r06/tail/): 512-1536 envs faster than the fused and split forms (C4 shard steady
// 13.3 -> 7.35 us, window 17.9 -> 15.3 us; 1536 envs window -3.4%), 2048 envs +4% and 4096 +24% in
// the window (the chip is full of physics waves, so the observation waits for the tail)
static constexpr int kTdmTailMaxEnvs = 2048;
static constexpr int kTdmSnapMinSteps = 32;  // the tail observation's first snapshot allocation, in steps
static bool tdm_tail_obs(macm_tdm* w) {
  const char* v = getenv("MACM_TDM_TAIL_OBS");
  if (v ? atoi(v) == 0 : w->P.n_envs >= kTdmTailMaxEnvs) return false;
  return tdm_tail_workers(w) >= 0;
}

// The steps observed in the tail: all below kTdmTailMaxEnvs; from there only the last
// MACM_TDM_TAIL_STEPS (the earlier steps observe in the step, the fused form), so that the observation
// of the last steps runs in the launch's tail while the heaviest envs finish
static int tdm_tail_k0(const macm_tdm* w, int n_steps) {
  int steps = w->P.n_envs >= kTdmTailMaxEnvs ? n_steps / 4 : n_steps;
  if (const char* v = getenv("MACM_TDM_TAIL_STEPS")) steps = atoi(v);
  if (steps < 1) steps = 1;
  if (steps > n_steps) steps = n_steps;
  return n_steps - steps;
}

// the tail observation's snapshot rows, grown rarely: a first allocation covers rollouts of up to
// kTdmSnapMinSteps steps, so that a short warm-up rollout does not leave the next, longer one a
// synchronising reallocation (macm_tdm_reserve sizes it ahead for longer ones)
static int tdm_tail_snapshots(macm_tdm* w, size_t rows, hipStream_t s) {
  if (rows <= w->tail_rows) return MACM_OK;
  const size_t E = w->P.n_envs, N = w->P.n_agents;
  const size_t want = rows > (size_t)kTdmSnapMinSteps * E ? rows : (size_t)kTdmSnapMinSteps * E;
  HIP_TRY(hipStreamSynchronize(s));
  if (w->tail_snap) HIP_TRY(hipFree(w->tail_snap));
  w->tail_snap = nullptr;
  w->tail_rows = 0;
  if (hipMalloc(&w->tail_snap, want * N * sizeof(float4)) != hipSuccess) {
    (void)hipGetLastError();
    w->tail_snap = nullptr;
    return fail(MACM_E_OOM, "hipMalloc (tail observation snapshots)");
  }
  w->tail_rows = want;
  return MACM_OK;
}

static int tdm_rollout_tail(macm_tdm* w, const TdmBuffers& TB, const void* actions, int n_steps,
                            const macm_tdm_outputs* out, hipStream_t s, unsigned long long astride) {
  const int k0 = tdm_tail_k0(w, n_steps);
  const size_t E = w->P.n_envs, rows = (size_t)(n_steps - k0) * E;
  if (!w->tail_ctl) {
    if (hipMalloc(&w->tail_ctl, tail_ctl_words((int)E) * sizeof(unsigned long long)) != hipSuccess) {
      (void)hipGetLastError();
      w->tail_ctl = nullptr;
      return fail(MACM_E_OOM, "hipMalloc (tail observation counters)");
    }
    HIP_TRY(hipMemsetAsync(w->tail_ctl, 0, tail_ctl_words((int)E) * sizeof(unsigned long long), s));
    w->tail_tag = 0;
  }
  if (const int rc = tdm_tail_snapshots(w, rows, s)) return rc;
  if (++w->tail_tag == 0) w->tail_tag = 1;  // tags are > 0: a ready word of 0 never matches
  TdmBuffers TBt = TB;
  TBt.snap_out = w->tail_snap;
  HIP_TRY(launch_tdm_rollout_w64(w->P, w->B, w->TP, TBt, w->cur, actions, out->obs, w->cfg.obs_f64 != 0, out->done, s,
                                 n_steps, astride, 1, w->tail_ctl, w->tail_tag, tdm_tail_workers(w), k0));
  if (n_steps & 1) w->cur ^= 1;
  return MACM_OK;
}

// A wave-kernel rollout (not the closed loop) with the split observation: the overwrite form keeps
// one snapshot row per env (the last step's) and observes it once; the trajectory form steps
// chunks of kTdmSplitChunk steps into alternating snapshot halves, each chunk observed on the
// observation stream while the caller's stream steps the next chunk.
static int tdm_rollout_split(macm_tdm* w, const TdmBuffers& TB, const void* actions, int n_steps,
                             const macm_tdm_outputs* out, hipStream_t s, unsigned long long astride, bool traj) {
  const size_t E = w->P.n_envs, N = w->P.n_agents, EN = E * N, S = N - 1;
  const bool f64 = w->cfg.obs_f64 != 0;
  const size_t orow = EN * S * 4 * (f64 ? sizeof(double) : sizeof(float));  // obs bytes per step
  if (!traj) {
    int rc = tdm_split_buffers(w, E, s);
    if (rc) return rc;
    TdmBuffers TBs = TB;
    TBs.snap_out = w->snap;
    HIP_TRY(launch_tdm_rollout_w64(w->P, w->B, w->TP, TBs, w->cur, actions, nullptr, f64, out ? out->done : nullptr, s,
                                   n_steps, astride, 0));
    if (n_steps & 1) w->cur ^= 1;
    HIP_TRY(launch_tdm_observe_snap(w->TP, (int)N, E, w->snap, out->obs, f64, TB.mask_out, s));
    return MACM_OK;
  }
  const int KC = n_steps < kTdmSplitChunk ? n_steps : kTdmSplitChunk;
  int rc = tdm_split_buffers(w, (size_t)KC * E, s);
  if (rc) return rc;
  const unsigned char* act = static_cast<const unsigned char*>(actions);
  unsigned char* obs = static_cast<unsigned char*>(out->obs);
  int c = 0;
  for (int k0 = 0; k0 < n_steps; k0 += KC, ++c) {
    const int kc = n_steps - k0 < KC ? n_steps - k0 : KC, b = c & 1;
    float4* snap = w->snap + (size_t)b * w->snap_rows * N;
    if (c >= 2) HIP_TRY(hipStreamWaitEvent(s, w->ev_obs[b], 0));  // chunk c - 2's observation has read this half
    TdmBuffers TBc = TB;
    auto row = [k0](auto* p, size_t per) { return p ? p + (size_t)k0 * per : p; };
    TBc.mask_out = nullptr;
    TBc.health_out = row(TB.health_out, EN);
    TBc.alive_out = row(TB.alive_out, EN);
    TBc.winner_out = row(TB.winner_out, E);
    TBc.snap_out = snap;
    HIP_TRY(launch_tdm_rollout_w64(w->P, w->B, w->TP, TBc, w->cur, act + (size_t)k0 * astride, nullptr, f64,
                                   row(out->done, E), s, kc, astride, 1));
    if (kc & 1) w->cur ^= 1;
    HIP_TRY(hipEventRecord(w->ev_phys[b], s));
    HIP_TRY(hipStreamWaitEvent(w->obs_stream, w->ev_phys[b], 0));
    HIP_TRY(launch_tdm_observe_snap(w->TP, (int)N, (size_t)kc * E, snap, obs ? obs + (size_t)k0 * orow : nullptr, f64,
                                    row(TB.mask_out, EN * S), w->obs_stream));
    HIP_TRY(hipEventRecord(w->ev_obs[b], w->obs_stream));
  }
  // joined: the caller's stream waits for the last chunk's observation (the stream is in order)
  HIP_TRY(hipStreamWaitEvent(s, w->ev_obs[(c - 1) & 1], 0));
  return MACM_OK;
}

// macm_tdm_rollout / _traj (bots = false) and macm_tdm_rollout_bots / _traj (bots = true)
static int tdm_rollout(macm_tdm* w, const void* actions, int n_steps, const macm_tdm_outputs* out, void* stream,
                       bool bots, bool traj) {
  if (n_steps < 0) return fail(MACM_E_INVALID, "n_steps must be >= 0");
  if (n_steps == 0) return MACM_OK;
  if (!w || !actions) return fail(MACM_E_INVALID, "tdm/actions is NULL");
  if ((bots || traj) && !out) return fail(MACM_E_INVALID, "out is NULL");
  if (bots && (!out->obs || !out->mask)) return fail(MACM_E_INVALID, "out->obs/mask is NULL (the bots act on them)");
  if (const uint32_t st = read_host_status(w->hstat)) return overflow_error(st);
  DeviceGuard g(w->device);
  hipStream_t s = (hipStream_t)stream;
  if (w->cfg.validate_actions) {
    // bots: the caller's first step, alive agents; else every agent's actions of every step, alive
    // or not (deaths are not known yet)
    const long long rows = (long long)(bots ? 1 : n_steps) * w->P.n_envs;
    if (rows > INT32_MAX) return fail(MACM_E_INVALID, "n_steps * n_envs too large to validate");
    const int rc =
        check_actions(w->bad, actions, 2, bots ? w->TB.alive : nullptr, (int)rows, w->P.n_agents, s, w->P.n_envs);
    if (rc) return rc;
  }
  const TdmBuffers TB = tdm_with_outputs(w, out);
  const unsigned long long astride = bots ? 0ull : (unsigned long long)w->P.n_envs * w->P.n_agents * 4;
  if (!w->wave) {
    // workgroup step (N > 64): one launch per step (and the bots kernel's), in order; trajectory
    // form: step k's outputs in row k of [K, ...], the closed loop reading action row k and the bot
    // writing row k + 1 of [K + 1, E, N, 4]
    const size_t E = w->P.n_envs, N = w->P.n_agents, EN = E * N;
    const size_t obytes = EN * (N - 1) * 4 * (w->cfg.obs_f64 ? sizeof(double) : sizeof(float));
    const unsigned long long kstride = bots ? (traj ? EN * 4 : 0ull) : astride;
    const unsigned char* act = static_cast<const unsigned char*>(actions);
    for (int k = 0; k < n_steps; ++k) {
      const size_t kr = traj ? (size_t)k : 0;
      TdmBuffers TBk = TB;
      auto row = [kr](auto* p, size_t per) { return p ? p + kr * per : p; };
      TBk.mask_out = row(TB.mask_out, EN * (N - 1));
      TBk.health_out = row(TB.health_out, EN);
      TBk.alive_out = row(TB.alive_out, EN);
      TBk.winner_out = row(TB.winner_out, E);
      void* obs_k = out && out->obs ? static_cast<unsigned char*>(out->obs) + kr * obytes : nullptr;
      const unsigned char* act_k = act + k * kstride;
      HIP_TRY(tdm_launch_step(w, TBk, w->cur, act_k, obs_k, out ? row(out->done, E) : nullptr, s));
      w->cur ^= 1;
      if (bots)
        HIP_TRY(launch_bots_combat(obs_k, TBk.mask_out, w->cfg.obs_f64 != 0, (int)N, (long long)EN,
                                   const_cast<unsigned char*>(act_k) + (traj ? EN * 4 : 0), s));
    }
    return MACM_OK;
  }
  if (!bots && traj && out && (out->obs || out->mask) && tdm_tail_obs(w))
    return tdm_rollout_tail(w, TB, actions, n_steps, out, s, astride);
  if (!bots && out && (out->obs || out->mask) && tdm_split_obs(w))
    return tdm_rollout_split(w, TB, actions, n_steps, out, s, astride, traj);
  HIP_TRY(launch_tdm_rollout_w64(w->P, w->B, w->TP, TB, w->cur, actions, out ? out->obs : nullptr,
                                 w->cfg.obs_f64 != 0, out ? out->done : nullptr, s, n_steps, astride, traj ? 1 : 0));
  if (n_steps & 1) w->cur ^= 1;
  return MACM_OK;
}

int macm_tdm_rollout(macm_tdm* w, const void* actions, int n_steps, const macm_tdm_outputs* out, void* stream) {
  return tdm_rollout(w, actions, n_steps, out, stream, false, false);
}

int macm_tdm_rollout_traj(macm_tdm* w, const void* actions, int n_steps, const macm_tdm_outputs* traj,
                          void* stream) {
  return tdm_rollout(w, actions, n_steps, traj, stream, false, true);
}

int macm_tdm_rollout_bots(macm_tdm* w, uint8_t* actions, int n_steps, const macm_tdm_outputs* out, void* stream) {
  return tdm_rollout(w, actions, n_steps, out, stream, true, false);
}

int macm_tdm_rollout_bots_traj(macm_tdm* w, uint8_t* actions, int n_steps, const macm_tdm_outputs* traj,
                               void* stream) {
  return tdm_rollout(w, actions, n_steps, traj, stream, true, true);
}

int macm_tdm_observe(macm_tdm* w, const macm_tdm_outputs* out, void* stream) {
  if (!w || !out) return fail(MACM_E_INVALID, "tdm/out is NULL");
  DeviceGuard g(w->device);
  const TdmBuffers TB = tdm_with_outputs(w, out);
  if (w->wave)
    HIP_TRY(launch_tdm_observe_w64(w->P, w->B, w->TP, TB, out->obs, w->cfg.obs_f64 != 0, (hipStream_t)stream));
  else
    HIP_TRY(launch_tdm_observe_wg(w->P, w->B, w->TP, TB, out->obs, w->cfg.obs_f64 != 0, (hipStream_t)stream));
  hipStream_t s = (hipStream_t)stream;
  const size_t EN = (size_t)w->P.n_envs * w->P.n_agents, E = (size_t)w->P.n_envs;
  if (out->health) HIP_TRY(hipMemcpyAsync(out->health, w->TB.health, EN * sizeof(double), hipMemcpyDefault, s));
  if (out->alive) HIP_TRY(hipMemcpyAsync(out->alive, w->TB.alive, EN, hipMemcpyDefault, s));
  if (out->done) HIP_TRY(hipMemcpyAsync(out->done, w->B.done, E, hipMemcpyDefault, s));
  if (out->winner) HIP_TRY(hipMemcpyAsync(out->winner, w->TB.winner, E * sizeof(int32_t), hipMemcpyDefault, s));
  return MACM_OK;
}

static int tdm_copy_state(macm_tdm* w, const macm_tdm_state* st, void* stream, bool to_device) {
  if (!w || !st) return fail(MACM_E_INVALID, "tdm/state is NULL");
  if (st->contact_stride < 0) return fail(MACM_E_INVALID, "contact_stride must be >= 0");
  DeviceGuard g(w->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t E = w->P.n_envs, N = w->P.n_agents, C = w->P.max_contacts;
  const size_t Cs = st->contact_stride > 0 ? (size_t)st->contact_stride : C;  // the caller's row length
  const size_t Cw = Cs < C ? Cs : C;                                           // entries moved per row
  struct Item {
    void* user;
    void* dev;
    size_t bytes;
  } items[] = {
      {st->pos, w->B.pos, E * N * sizeof(float2)},
      {st->vel, w->B.vel, E * N * sizeof(float2)},
      {st->angle, w->B.angle, E * N * sizeof(float)},
      {st->fat, w->B.fat, E * N * sizeof(float4)},
      {st->sleep, w->B.sleep, E * N * sizeof(float)},
      {st->health, w->TB.health, E * N * sizeof(double)},
      {st->cd_atk, w->TB.cd_atk, E * N * sizeof(double)},
      {st->cd_mov, w->TB.cd_mov, E * N * sizeof(double)},
      {st->alive, w->TB.alive, E * N},
      {st->listener, w->TB.listener, E * sizeof(int2)},
      {st->step_count, w->B.step_count, E * sizeof(int32_t)},
      {st->time_passed, w->B.time_passed, E * sizeof(double)},
      {st->done, w->B.done, E},
      {st->winner, w->TB.winner, E * sizeof(int32_t)},
  };
  if (!to_device) {
    if (st->contact_count)
      HIP_TRY(hipMemcpyAsync(st->contact_count, w->B.ccount[w->cur], E * sizeof(int32_t), hipMemcpyDefault, s));
    if (st->contact_ab)
      HIP_TRY(copy_rows(st->contact_ab, Cs * sizeof(uint32_t), w->B.cab[w->cur], C * sizeof(uint32_t),
                        Cw * sizeof(uint32_t), E, s));
    if (st->contact_imp)
      HIP_TRY(copy_rows(st->contact_imp, Cs * sizeof(float2), w->B.cimp[w->cur], C * sizeof(float2),
                        Cw * sizeof(float2), E, s));
  }
  if (to_device) {
    if (!st->contact_count != !st->contact_ab)
      return fail(MACM_E_INVALID, "contact_count and contact_ab must be given together");
    if (st->contact_count) {
      const int rc = stage_lists(w->B, w->cur, w->bad, E, C, Cs, (int)N, st->contact_count, st->contact_ab,
                                 st->contact_imp, s);
      if (rc) return rc;
      w->cur ^= 1;
    }
    HIP_TRY(hipStreamSynchronize(s));
    clear_host_status(w->hstat);
    HIP_TRY(hipMemsetAsync(w->B.status, 0, E * sizeof(int32_t), s));
  }
  for (const Item& it : items) {
    if (!it.user) continue;
    if (to_device) HIP_TRY(hipMemcpyAsync(it.dev, it.user, it.bytes, hipMemcpyDefault, s));
    else HIP_TRY(hipMemcpyAsync(it.user, it.dev, it.bytes, hipMemcpyDefault, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return MACM_OK;
}

int macm_tdm_get_state(macm_tdm* w, const macm_tdm_state* dst, void* stream) {
  return tdm_copy_state(w, dst, stream, false);
}

int macm_tdm_set_state(macm_tdm* w, const macm_tdm_state* src, void* stream) {
  return tdm_copy_state(w, src, stream, true);
}

int macm_tdm_status(macm_tdm* w, int32_t* status_or, void* stream) {
  if (!w || !status_or) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  std::vector<int32_t> st(w->P.n_envs);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(st.data(), w->B.status, st.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  int32_t acc = 0;
  for (int32_t v : st) acc |= v;
  *status_or = acc;
  return MACM_OK;
}

int macm_tdm_counters(macm_tdm* w, int64_t out[4], void* stream) {
  if (!w || !out) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  std::vector<unsigned long long> h((size_t)w->P.n_envs * 4);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(h.data(), w->B.env_counters, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                         s));
  HIP_TRY(hipStreamSynchronize(s));
  unsigned long long acc[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < h.size(); ++i) acc[i & 3] += h[i];
  for (int i = 0; i < 4; ++i) out[i] = (int64_t)acc[i];
  return MACM_OK;
}

int macm_tdm_launch_flags(const macm_tdm* w) {
  if (!w) return fail(MACM_E_INVALID, "tdm is NULL");
  return (tdm_split_obs(w) ? MACM_LAUNCH_SPLIT_OBS : 0) |
         (tdm_tail_obs(const_cast<macm_tdm*>(w)) ? MACM_LAUNCH_TAIL_OBS : 0);
}

int macm_tdm_reserve(macm_tdm* w, int32_t n_steps, void* stream) {
  if (!w || n_steps < 0) return fail(MACM_E_INVALID, "tdm is NULL or n_steps < 0");
  DeviceGuard g(w->device);
  if (!tdm_tail_obs(w) || n_steps == 0) return MACM_OK;
  const int k0 = tdm_tail_k0(w, n_steps);
  return tdm_tail_snapshots(w, (size_t)(n_steps - k0) * w->P.n_envs, (hipStream_t)stream);
}

int macm_tdm_spilled(macm_tdm* w, int64_t* env_steps, void* stream) {
  if (!w || !env_steps) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  std::vector<uint32_t> h((size_t)w->P.n_envs);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(h.data(), w->B.spill_count, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  int64_t acc = 0;
  for (uint32_t v : h) acc += v;
  *env_steps = acc;
  return MACM_OK;
}

int macm_tdm_set_debug(macm_tdm* w, int32_t flags) {
  if (!w) return fail(MACM_E_INVALID, "world is NULL");
  const int pool = (flags & MACM_DEBUG_SPILL_POOL) ? (flags >> 8) : 0;
  flags &= 0xff;
  if (flags & ~(MACM_DEBUG_FORCE_SPILL | MACM_DEBUG_SPILL_POOL | MACM_DEBUG_SPILL_FAIL))
    return fail(MACM_E_INVALID, "unknown debug flag (TDM: FORCE_SPILL, SPILL_POOL, SPILL_FAIL)");
  if (int rc = set_spill_pool(w, flags, pool)) return rc;
  w->P.force_spill = (flags & MACM_DEBUG_FORCE_SPILL) ? 1 : 0;
  return MACM_OK;
}

// ============================ scripted actors ===============================

int macm_bots_flock(const void* obs, int32_t obs_f64, int32_t obs_dim, int64_t rows, uint8_t* actions,
                    void* stream) {
  if (!obs || !actions || rows < 0) return fail(MACM_E_INVALID, "obs/actions NULL or rows < 0");
  if (obs_dim != 4 && obs_dim != 6) return fail(MACM_E_INVALID, "obs_dim must be 4 (polar) or 6 (cartesian)");
  HIP_TRY(launch_bots_flock(obs, obs_f64 != 0, obs_dim, rows, actions, (hipStream_t)stream));
  return MACM_OK;
}

int macm_bots_combat(const void* obs, const uint8_t* mask, int32_t obs_f64, int32_t n_agents, int64_t rows,
                     uint8_t* actions, void* stream) {
  if (!obs || !mask || !actions || rows < 0) return fail(MACM_E_INVALID, "obs/mask/actions NULL or rows < 0");
  if (n_agents < 2) return fail(MACM_E_INVALID, "n_agents must be >= 2");
  HIP_TRY(launch_bots_combat(obs, mask, obs_f64 != 0, n_agents, rows, actions, (hipStream_t)stream));
  return MACM_OK;
}

#ifdef MACM_STAMPS
// Diagnostic build only: copy the per-env phase stamps [E, 32] of the last step (the wave kernel
// uses rows of 16).
int macm_debug_stamps(macm_world* w, unsigned long long* out) {
  if (!w || !out) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  HIP_TRY(hipMemcpy(out, w->B.stamps, (size_t)w->P.n_envs * 32 * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
  return MACM_OK;
}
int macm_debug_tdm_stamps(macm_tdm* w, unsigned long long* out) {
  if (!w || !out) return fail(MACM_E_INVALID, "NULL argument");
  DeviceGuard g(w->device);
  HIP_TRY(hipMemcpy(out, w->B.stamps, (size_t)w->P.n_envs * 32 * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
  return MACM_OK;
}
#endif

}  // extern "C"
