/*
 * macm.h — C-ABI of the MI355X-native batched gym-macm stepper (libmacm_hip.so).
 *
 * What this replaces (reference = siyarvurucu/gym-macm, file:line):
 *   - the per-env Box2D world owned by FrameworkBase
 *       gym_macm/cm_framework.py:155-167  (b2World(gravity=(0,0), doSleep=True))
 *       gym_macm/backends/no_render.py:4-19 (NoRender, the headless framework)
 *   - the body construction loop of Flock.__init__      gym_macm/envs/mvmnt.py:35-79
 *   - the whole env.step hot path                        gym_macm/envs/mvmnt.py:81-140
 *       action -> angle/force (:97-129), FrameworkBase.Step -> b2World.Step(1/60,8,3)
 *       + ClearForces (cm_framework.py:172-225), get_rewards (:160-179),
 *       time/done (:134-136), get_obs (:181-222)
 *
 * The reference's "API" at this boundary is pybox2d (SWIG) called per agent from
 * Python. Here one call advances E independent envs of N agents each, with all
 * per-agent arrays on the device (SoA), so control crosses host->device once per
 * step. No torch / C++ types cross this ABI: plain pointers, sizes, POD structs.
 *
 * Conventions
 *   - Every function returns int status: MACM_OK (0) or a negative MACM_E_* code;
 *     macm_last_error() returns a thread-local message for the last failure.
 *     Nothing aborts or throws across the ABI.
 *   - "device pointer" = memory the HIP runtime can dereference in a kernel
 *     (hipMalloc / torch CUDA tensor data_ptr()). Output buffers are borrowed for
 *     the duration of the call only; the world owns its state.
 *   - stream = hipStream_t passed as void* (NULL = default stream). Calls are
 *     asynchronous on that stream; completion is the caller's synchronisation.
 *   - A world is bound to one device. Calls on one world are not thread-safe.
 */
#ifndef MACM_H
#define MACM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MACM_ABI_VERSION 9

enum {
  MACM_OK = 0,
  MACM_E_INVALID = -1,     /* bad argument / config / action (validate_actions) */
  MACM_E_OOM = -2,         /* device allocation failed                       */
  MACM_E_HIP = -3,         /* HIP runtime error                              */
  MACM_E_UNSUPPORTED = -4, /* config valid for the reference, not built here */
  MACM_E_OVERFLOW = -5     /* a per-env capacity overflowed in an earlier step: results since
                              then are not the reference's (reset / place / set_state clear it) */
};

enum { MACM_ACTION_DISCRETE = 0, MACM_ACTION_CONTINUOUS = 1 };
enum { MACM_REWARD_BINARY = 0, MACM_REWARD_LINEAR = 1 };
enum { MACM_COORD_POLAR = 0, MACM_COORD_CARTESIAN = 1 };

/*
 * Status bits accumulated per env on the device (macm_world_status). TOUCH/DEGREE are no longer
 * set (ABI 6): an env of either kind whose touching contacts exceed a fast kernel's LDS capacity
 * is stepped by the spill step (HBM working set sized by max_contacts) instead. CONTACT_OVERFLOW
 * (the fat-AABB pair list itself outgrew max_contacts; never for TDM, whose list holds every
 * pair) and SPILL_WAIT remain. Detection
 * is eventual, not synchronous: the kernels store the bits into a host-mapped word, and each step /
 * rollout call reads it before launching, without synchronising, so steps already queued behind an
 * overflowing one still run (and a rollout keeps stepping the overflowed env for its K steps); the
 * first call that sees the word returns MACM_E_OVERFLOW. macm_world_status() (which synchronises)
 * is exact. reset / place / set_state clear the bits; reset_envs re-derives the word from the envs
 * it did not reset.
 */
enum {
  MACM_ST_CONTACT_OVERFLOW = 1, /* Ov(F_t) list exceeded max_contacts                   */
  MACM_ST_TOUCH_OVERFLOW = 2,   /* (before ABI 6) TDM touching contacts beyond capacity  */
  MACM_ST_DEGREE_OVERFLOW = 4,  /* (before ABI 6) TDM body degree beyond capacity        */
  MACM_ST_INVALID_ACTION = 8,   /* validate_actions: an action outside the action space  */
  MACM_ST_SPILL_WAIT = 16,      /* a dense env found no free spill working-set slot for ~1 s
                                   (a pooled world: fewer slots than envs) and was not stepped */
  MACM_ST_HANDOFF = 32          /* workgroup path: kernel B's waves did not all start within ~1 s
                                   of B's dependencies finishing, or a kernel-C block waited ~1 s
                                   for B to hand it an env and skipped it (never expected: B's
                                   waves wait for nothing). Every env of the world carries the bit
                                   (the skipped env is unknown); results since then are invalid
                                   (ABI 8)                                                      */
};

/* macm_world_set_debug / macm_tdm_set_debug flags (test hooks; 0 = product behaviour; TDM takes
 * FORCE_SPILL, SPILL_POOL and SPILL_FAIL). */
enum {
  MACM_DEBUG_FORCE_SPILL = 1,     /* every env takes the spill step (parity tests of that path)  */
  MACM_DEBUG_SWEEP_CELLS = 2,     /* N > 64: pair sweep over strip cells at any N (else N >= 256) */
  MACM_DEBUG_SWEEP_ALL_PAIRS = 4, /* N > 64: all-pairs pair sweep at any N                        */
  MACM_DEBUG_SPILL_POOL = 8,      /* the spill working set as a pool of (flags >> 8) slots, at most
                                     the slots allocated (pooled-slot tests at small E)            */
  MACM_DEBUG_SPILL_FAIL = 16      /* no spill slot is ever free: every env that needs the spill step
                                     is left unstepped with MACM_ST_SPILL_WAIT (ABI 8 test hook)   */
};

/*
 * macm_config — flockSettings (gym_macm/settings.py:110-146) + fwSettings
 * (settings.py:25-59) flattened. Field names follow the reference's attribute
 * names. macm_config_default() fills the reference defaults.
 */
typedef struct macm_config {
  int32_t n_agents;            /* sum(n_agents)                     mvmnt.py:61      */
  int32_t n_targets;           /* len(np.unique(targets))           mvmnt.py:42      */
  int32_t action_mode;         /* "discrete"/"continuous"           settings.py:136  */
  int32_t reward_mode;         /* "binary"/"linear"                 settings.py:137  */
  int32_t coord;               /* "polar"/"cartesian"               settings.py:141  */
  int32_t velocity_iterations; /* 8                                 settings.py:31   */
  int32_t position_iterations; /* 3                                 settings.py:32   */
  int32_t warm_starting;       /* enableWarmStarting = True         settings.py:34   */
  int32_t obs_f64;             /* 0: obs written as float32, 1: float64              */
  int32_t validate_actions;    /* 1: macm_world_step checks every action against the
                                  action space first (assert action_space.contains,
                                  mvmnt.py:94) and returns MACM_E_INVALID without
                                  stepping; synchronises the stream. 0 (default): no check */
  double hz;                   /* 60.0                              settings.py:30   */
  double start_spread;         /* 20                                settings.py:119  */
  double start_point[2];       /* [0, 0]                            settings.py:120  */
  double agent_rotation_speed; /* 0.8 * 2pi                         settings.py:121  */
  double agent_force;          /* 20                                settings.py:122  */
  double time_limit;           /* 60                                settings.py:123  */
  double reward_radius;        /* 7 if binary else 1                settings.py:146  */
  double target_mindist;       /* 25                                settings.py:139  */
  double target_maxdist;       /* 60                                settings.py:140  */
  float radius;                /* circle r = 0.5                    settings.py:127-131 */
  float density;               /* 1                                                  */
  float friction;              /* 0.3                                                */
  float linear_damping;        /* 5                                 settings.py:133  */
} macm_config;

/*
 * macm_tdm_config — the team-deathmatch env (gym_macm/envs/combat.py:13-264,
 * combatSettings settings.py:149-177). The reference's TDM cannot be built as
 * shipped (combat.py:65 NameError; :150-151,173 read attributes that do not
 * exist); this is its semantics with those four names supplied from
 * combatSettings, everything else literal (see DESIGN.md "TDM").
 */
typedef struct macm_tdm_config {
  int32_t n_teams;              /* len(n_agents)                      combat.py:70-73 */
  int32_t team_size[4];         /* n_agents[i]                                        */
  int32_t n_agents;             /* sum(n_agents) (<= 4096; > 64: the workgroup step)   */
  int32_t velocity_iterations;  /* 8                                                  */
  int32_t position_iterations;  /* 3                                                  */
  int32_t warm_starting;        /* 1                                                  */
  int32_t obs_f64;              /* obs written as float32 (0) or float64 (1)          */
  int32_t fresh_raycast;        /* 0 (reference): ONE RayCastClosestCallback whose hit /
                                   fixture are never reset (cm_framework.py:62-65,76,
                                   combat.py:147-153), so after the first hit every
                                   attack damages the last-hit body. 1: per-cast hit.  */
  int32_t decay_mov_penalty;    /* 0 (reference): cooldown_mov_penalty is never
                                   decremented (combat.py:151,155). 1: decremented by
                                   1/hz alongside cooldown_atk.                        */
  int32_t validate_actions;     /* 1: macm_tdm_step checks the alive agents' actions
                                   (assert action_space.contains, combat.py:118) first,
                                   MACM_E_INVALID without stepping; synchronises          */
  int32_t _pad;
  double hz;                    /* 60                                                 */
  double world_width;           /* 30                                 combat.py:76    */
  double world_height;          /* 30                                 combat.py:77    */
  double agent_rotation_speed;  /* 0.8 * 2pi                          combat.py:18    */
  double agent_force;           /* 20                                 combat.py:19    */
  double percent_mov_penalty;   /* 0.2                                combat.py:22    */
  double melee_range;           /* 2                                  combat.py:20    */
  double melee_dmg;             /* 0.25                               combat.py:21    */
  double init_health;           /* 1                                  combat.py:14    */
  double cooldown_atk;          /* 1                                  settings.py:164 */
  double cooldown_mov_penalty;  /* 0.5                                settings.py:165 */
  double time_limit;            /* 60                                 settings.py:163 */
  float radius, density, friction, linear_damping;
} macm_tdm_config;

/*
 * Device-side outputs of one TDM step (device pointers; NULL = not wanted).
 * TDM.get_obs (combat.py:206-227) as fixed slots: slot k of agent i is agent
 * j = k < i ? k : k + 1 and holds (r, t, p, is_ally); the dict API lists the alive
 * j in the same order. mask = agents i and j both alive; masked slots are zero.
 */
typedef struct macm_tdm_outputs {
  void* obs;        /* [E, N, N-1, 4] float32 or float64 (config.obs_f64)     */
  uint8_t* mask;    /* [E, N, N-1]                                           */
  double* health;   /* [E, N]  Agent.health                                  */
  uint8_t* alive;   /* [E, N]  Agent.alive                                   */
  uint8_t* done;    /* [E]     TDM.done (latches)                            */
  int32_t* winner;  /* [E]     TDM.winner, -1 = None                         */
} macm_tdm_outputs;

/*
 * TDM state, SoA (host or device pointers, NULL = skip). Physics fields as
 * macm_state; plus
 *   health, cd_atk, cd_mov [E, N] float64   Agent.health / cooldown_atk / cooldown_mov_penalty
 *   alive                  [E, N] uint8
 *   listener               [E, 2] int32     (RayCastClosestCallback.hit, body of .fixture or -1)
 *   done [E] uint8, winner [E] int32
 *   contact_stride         entries per env row of the caller's contact_ab / contact_imp, as
 *                          macm_state (0 = C = N(N-1)/2; ABI 7: a stride of max(contact_count)
 *                          moves only the lists' used part, C is 523,776 at N = 1024)
 */
typedef struct macm_tdm_state {
  void* pos;
  void* vel;
  void* angle;
  void* fat;
  void* sleep;
  void* health;
  void* cd_atk;
  void* cd_mov;
  void* alive;
  void* listener;
  void* contact_count;
  void* contact_ab;
  void* contact_imp;
  void* step_count;
  void* time_passed;
  void* done;
  void* winner;
  int64_t contact_stride;
} macm_tdm_state;

/*
 * Device-side outputs of one step (all device pointers; NULL = not wanted,
 * except reward which is required). Shapes: E = n_envs, N = n_agents,
 * OD = 4 (polar: nbr r, nbr t, target r, target t) or 6 (cartesian: nbr r,
 * cos t, sin t, target r, cos t, sin t). Matches Flock.get_obs node order
 * (mvmnt.py:197-220): node 0 = closest agent (type 0, id = nbr_id), node 1 =
 * the agent's target (type 1, id = N).
 */
typedef struct macm_outputs {
  void* obs;        /* [E, N, OD] float32 or float64 (config.obs_f64)          */
  int32_t* nbr_id;  /* [E, N] index of the closest other agent                 */
  float* reward;    /* [E, N] -1 in any contact, else binary 0/1 or linear     */
  uint8_t* collided;/* [E, N] 1 if the agent is in world.contacts              */
  uint8_t* done;    /* [E] time_passed > time_limit                            */
} macm_outputs;

/*
 * World state, SoA. Used by get/set_state (parity injection, checkpoints).
 * Pointers may be host or device memory (copied with hipMemcpyDefault).
 *   pos, vel      [E, N, 2] float32   body position (sweep c) / linear velocity
 *   angle         [E, N]    float32   sweep angle
 *   fat           [E, N, 4] float32   broad-phase fat AABB (lo.x, lo.y, hi.x, hi.y)
 *   sleep         [E, N]    float32   sleepTime
 *   targets       [E, T, 2] float32
 *   contact_count [E]       int32     length of the ordered contact list
 *   contact_ab    [E, C]    uint32    a | b << 16, a < b, Box2D world-list order
 *   contact_imp   [E, C, 2] float32   (normalImpulse, tangentImpulse) warm start
 *   step_count    [E]       int32     steps taken (0 => dtRatio 0 on next step)
 *   time_passed   [E]       float64
 *   contact_stride            entries per env row of the caller's contact_ab / contact_imp
 *                             (0 = C = macm_world_info().max_contacts). get_state fills the first
 *                             min(stride, C) entries of each row: a stride of max(contact_count)
 *                             moves only the lists' used part (ABI 5; C can be large for N > 64).
 */
typedef struct macm_state {
  void* pos;
  void* vel;
  void* angle;
  void* fat;
  void* sleep;
  void* targets;
  void* contact_count;
  void* contact_ab;
  void* contact_imp;
  void* step_count;
  void* time_passed;
  int64_t contact_stride;
} macm_state;

typedef struct macm_world_info {
  int32_t n_envs, n_agents, n_targets, obs_dim;
  int32_t max_contacts;   /* per-env ordered contact list capacity */
  int32_t max_touching;   /* per-env solver capacity               */
  int32_t device;
  int32_t spill_slots;    /* spill working-set slots (= n_envs: one per env; fewer: a pool) */
  int32_t launch_flags;   /* MACM_LAUNCH_* of the workgroup step, decided at the first step (ABI 8) */
  int32_t rollout_slices; /* env slices a workgroup-path rollout runs on streams of their own (0: none;
                             MACM_WG_SLICES overrides the default 3) (ABI 9)                       */
} macm_world_info;

/* macm_world_info.launch_flags */
#define MACM_LAUNCH_HANDOFF 1  /* kernel C as kernel B's consumer on a second stream (MACM_HANDOFF) */
#define MACM_LAUNCH_SPLIT_OBS 2 /* TDM (macm_tdm_launch_flags, ABI 9): the step writes pose snapshots and
                                   tdm_observe_snap observes them in a launch of its own (fewer than
                                   1024 envs, N <= 64; MACM_TDM_SPLIT_OBS overrides); same results */
#define MACM_LAUNCH_TAIL_OBS 4  /* TDM trajectory rollouts (macm_tdm_rollout_traj): the tail observation,
                                   each env's wave steps its K steps writing pose snapshots, then the
                                   finished waves and observe-only waves observe the (step, env) rows
                                   (fewer than 2048 envs, N <= 64, the launch resident at once;
                                   MACM_TDM_TAIL_OBS overrides); same results */

typedef struct macm_world macm_world;

/* Library identity. */
const char* macm_version(void);
int macm_abi_version(void);
const char* macm_last_error(void);

/* Reference defaults (settings.py:25-59, 110-146). */
int macm_config_default(macm_config* cfg);

/*
 * Create E envs of one Flock configuration on `device`.
 *   targets_idx: host int32[N], agent -> target index (mvmnt.py:43), or NULL = all 0.
 *   max_contacts: per-env capacity C of the ordered fat-AABB pair list (and of each slot of
 *   the spill step's HBM working set). 0 = the default, from a budget of 1/8 of the device's
 *   free memory at creation (so every world shrinks what the next one sees), half for the lists
 *   (24 B per entry and env): N(N-1)/2 (every pair: the list can never overflow) when N <= 64 or
 *   when that fits, otherwise the largest C that fits (at least 32 N). The other half holds the
 *   spill working set, 48 B per entry and 48 B per body per slot: one slot per env when they fit,
 *   otherwise a pool (>= 16 slots) that dense envs take turns on (macm_world_info: spill_slots).
 *   On an idle 288 GB MI355X: C5's shard (2048 envs x 1024 agents) gets C ~ 366k and ~1k slots.
 *   Overflow of the list sets MACM_ST_CONTACT_OVERFLOW and a later step returns MACM_E_OVERFLOW.
 * Replaces: Flock.__init__ world + body creation (mvmnt.py:35-79,
 * cm_framework.py:155-167). State is undefined until macm_world_reset.
 */
int macm_world_create(const macm_config* cfg, const int32_t* targets_idx, int32_t n_envs,
                      int32_t device, int32_t max_contacts, macm_world** out);
int macm_world_destroy(macm_world* w);
int macm_world_info_get(const macm_world* w, macm_world_info* info);

/*
 * Initialise every env exactly as Flock.__init__ would after
 * random.seed(seed + env_offset + e) (CPython MT19937; mvmnt.py:47-79 draw order:
 * targets (angle, dist) then agents (x, y, angle)). Resets time, contacts, status.
 * Writes the initial observation (Flock.obs, mvmnt.py:79) into `out` if non-NULL.
 */
int macm_world_reset(macm_world* w, uint64_t seed, int64_t env_offset, const macm_outputs* out,
                     void* stream);

/*
 * Like macm_world_reset, but with caller-drawn poses (host or device pointers):
 * pos [E, N, 2] float32, angle [E, N] float32, targets [E, T, 2] float32. Used by
 * the drop-in Flock facade, which draws them from Python's global `random` in
 * the reference's order (mvmnt.py:47-64) so the caller's RNG stream advances
 * exactly as the reference's would.
 */
int macm_world_place(macm_world* w, const void* pos, const void* angle, const void* targets,
                     const macm_outputs* out, void* stream);

/*
 * Start a new episode in the envs selected by env_mask (device or host uint8 [E],
 * nonzero = reset; NULL = all), e.g. the done flags of the last step. Each env
 * continues the CPython MT19937 stream macm_world_reset seeded it with, drawing
 * the next agent poses exactly as the reference's reset() draws them from the
 * global `random` (mvmnt.py:224-233, targets kept); velocities, sleep clocks,
 * contacts, time and done restart. The new episodes' initial obs are written into
 * `out` for the reset envs only. Asynchronous on `stream` (no host round trip).
 * Fails with MACM_E_INVALID after macm_world_place (no device streams).
 */
int macm_world_reset_envs(macm_world* w, const uint8_t* env_mask, const macm_outputs* out, void* stream);

/*
 * One env.step for all E envs.
 *   actions: device pointer. Discrete: uint8/int8 [E, N, 3] in {0,1,2}
 *   (MultiDiscrete([3,3,3]), mvmnt.py:143-145). Continuous: float32 [E, N, 2] in [-1,1].
 * Replaces Flock.step (mvmnt.py:81-140) incl. b2World.Step(1/hz, 8, 3) + ClearForces.
 * Returns MACM_E_OVERFLOW (and launches nothing) if an earlier step or reset set a status bit
 * (read from a host-mapped word the kernels write; no synchronisation). With
 * cfg.validate_actions, returns MACM_E_INVALID and steps no env if any action is outside the
 * action space (reference: AssertionError before any agent acts, mvmnt.py:94).
 */
int macm_world_step(macm_world* w, const void* actions, const macm_outputs* out, void* stream);

/*
 * n_steps consecutive env.steps of all E envs with actions given in advance, e.g. the
 * reference's random-action loop (`env.step(env.action_space.sample())`, mvmnt.py:271-293),
 * in one launch on the wave path (N <= 64): each env's wave runs its steps back to back, so no
 * env waits at a launch boundary for the slowest env of the batch. Results are those of
 * n_steps macm_world_step calls with the same actions.
 *   actions: device pointer, [n_steps, E, N, 3] uint8 (discrete) or [n_steps, E, N, 2] float32.
 *   out: overwritten by every step; the last step's outputs remain. Counters accumulate all steps.
 * The workgroup path (N > 64) launches its steps one after another. n_steps = 0 does nothing
 * (actions may then be NULL).
 * With cfg.validate_actions every step's actions are checked before any env is stepped.
 */
int macm_world_rollout(macm_world* w, const void* actions, int32_t n_steps, const macm_outputs* out, void* stream);

/*
 * n_steps of the closed loop `step -> bots.flock -> step` (test_scripts/bots.py:37-61 acting on every
 * agent's observation, as macm_bots_flock) in one launch on the wave path: each env's wave steps,
 * then every lane takes its agent's next action from the observation just written.
 *   actions: device uint8 [E, N, 3]; in: the first step's actions (e.g. macm_bots_flock on the
 *   initial obs); out: the bot's actions for the step after the last. out->obs must be set.
 * Same results as n_steps of (macm_world_step, macm_bots_flock). Workgroup path: those launches.
 */
int macm_world_rollout_bots(macm_world* w, uint8_t* actions, int32_t n_steps, const macm_outputs* out, void* stream);

/*
 * Trajectory forms: as macm_world_rollout / macm_world_rollout_bots, but every step's outputs are
 * kept, as the reference returns (obs, rewards) from every env.step (mvmnt.py:140): each non-NULL
 * field of `traj` is a [n_steps, ...] buffer whose row k receives step k's outputs
 * (obs [n_steps, E, N, OD], nbr_id / reward / collided [n_steps, E, N], done [n_steps, E]).
 * Bots form: actions is [n_steps + 1, E, N, 3]; row 0 holds the first step's actions on entry and
 * step k writes the bot's actions for step k + 1 into row k + 1, so (obs, action, reward) of every
 * step stay in HBM. Same results as the per-step calls; one launch on the wave path (ABI 5).
 */
int macm_world_rollout_traj(macm_world* w, const void* actions, int32_t n_steps, const macm_outputs* traj,
                            void* stream);
int macm_world_rollout_bots_traj(macm_world* w, uint8_t* actions, int32_t n_steps, const macm_outputs* traj,
                                 void* stream);

/* Observation of the current state without stepping (Flock.get_obs, mvmnt.py:181-222). */
int macm_world_observe(macm_world* w, const macm_outputs* out, void* stream);

/*
 * Copy state out / in (synchronous w.r.t. `stream`). set_state validates the contact lists
 * it is given (when contact_count is non-NULL): 0 <= count <= min(C, contact_stride) and, for
 * every entry below the count, a < b < N, checked on the device after staging the lists into the
 * world's spare list buffer; otherwise MACM_E_INVALID and nothing is copied. contact_count and
 * contact_ab must be given together (contact_imp NULL: zero impulses). Clears the status bits.
 */
int macm_world_get_state(macm_world* w, const macm_state* dst, void* stream);
int macm_world_set_state(macm_world* w, const macm_state* src, void* stream);

/* OR over envs of the per-env status bits (synchronises `stream`). */
int macm_world_status(macm_world* w, int32_t* status_or, void* stream);

/*
 * Per-world counters, accumulated on device by every step (synchronises `stream`):
 *   out[0] agent-steps, out[1] collided agent-steps, out[2] positive-reward
 *   agent-steps, out[3] env-steps with done set. Used for the RCCL all-reduce
 *   in multi-GPU runs. reset_counters zeroes them.
 */
int macm_world_counters(macm_world* w, int64_t out[4], void* stream);
int macm_world_reset_counters(macm_world* w, void* stream);  /* also zeroes the reward sums */

/*
 * The rewards' sum (Σ of get_rewards' values, mvmnt.py:160-179), in float64 and
 * in a fixed order so that it is bit-stable (ABI 8): each step's float32 rewards are summed as
 * float64 pairwise over the agent slots 0 .. P-1 (P = 64 * 2^ceil(log2(ceil(N / 64))), +0.0 past N:
 * ((r0 + r1) + (r2 + r3)) + ...), that sum is added to the env's total in step order, and `total`
 * is the envs' totals summed in env order from +0.0. Binary rewards (-1, 0, +1) make every partial sum
 * an exact integer, so a binary world's env total is read as counter 2 - counter 1 (the same bits; the
 * kernels accumulate the float64 sums for linear rewards only). per_env: host double [E] or NULL; total: host
 * double or NULL (not both NULL). Accumulated by every step since creation or reset_counters;
 * synchronises `stream`. Multi-GPU: gather the per-env totals and sum them in global env order
 * (gym_macm.dist.reduce_reward_sums), which gives the single-process total at any rank count.
 */
int macm_world_reward_sums(macm_world* w, double* per_env, double* total, void* stream);

/* Env-steps taken by the spill step since creation (dense worlds; synchronises `stream`). */
int macm_world_spilled(macm_world* w, int64_t* env_steps, void* stream);

/* Test hooks: MACM_DEBUG_* flags (0 = product behaviour). */
int macm_world_set_debug(macm_world* w, int32_t flags);

/* ---- TDM (gym_macm:cm-tdm-v0, combat.py:57-264) -------------------------- */

typedef struct macm_tdm macm_tdm;

/* combatSettings / Agent defaults (settings.py:149-177, combat.py:13-29), n_agents=[1,1]. */
int macm_tdm_config_default(macm_tdm_config* cfg);

/*
 * Create E TDM envs (N = sum(team_size) <= 4096 agents; MACM_E_UNSUPPORTED above). Replaces
 * TDM.__init__'s world + body creation (combat.py:61-102). State is undefined until reset/place.
 * N <= 64: one wave per env (the fast kernel, its spill step for crowded envs); N > 64: one
 * workgroup per env (tdm_step_wg.hip: the action loop, then the spill step's physics with its HBM
 * working set for every env; macm_tdm_spilled counts every such env-step). Rollouts on the
 * workgroup path are one launch per step (and the bots kernel's), with the same results.
 */
int macm_tdm_create(const macm_tdm_config* cfg, int32_t n_envs, int32_t device, macm_tdm** out);
int macm_tdm_destroy(macm_tdm* w);

/*
 * Initialise every env as TDM.__init__ after random.seed(seed + env_offset + e):
 * per agent in team order x = random()*(team + width/2), y = random()*height,
 * angle = uniform(-1, 1)*pi (combat.py:80-95). Writes the initial obs into `out`.
 */
int macm_tdm_reset(macm_tdm* w, uint64_t seed, int64_t env_offset, const macm_tdm_outputs* out, void* stream);

/* As reset with caller-drawn poses: pos [E, N, 2] float32, angle [E, N] float32. */
int macm_tdm_place(macm_tdm* w, const void* pos, const void* angle, const macm_tdm_outputs* out, void* stream);

/*
 * As macm_world_reset_envs for TDM: the masked envs draw new spawn poses from
 * their streams (combat.py:234-245 draw order), every agent revived with
 * init_health, zero cooldowns, a fresh listener, winner -1.
 */
int macm_tdm_reset_envs(macm_tdm* w, const uint8_t* env_mask, const macm_tdm_outputs* out, void* stream);

/*
 * One TDM.step for all E envs (combat.py:104-184). actions: device uint8
 * [E, N, 4] (MultiDiscrete([3,3,3,2]): forward, lateral, rotation, attack);
 * rows of dead agents are ignored. An env with more than 256 touching contacts or a body touching
 * more than 16 others (a crowded small world) is stepped by the spill step (HBM working set,
 * every pair; after its actions, casts and deaths) with the same results. MACM_E_INVALID with
 * validate_actions; MACM_E_OVERFLOW only after a SPILL_WAIT (pooled working set).
 */
int macm_tdm_step(macm_tdm* w, const void* actions, const macm_tdm_outputs* out, void* stream);

/*
 * As macm_world_rollout for TDM: actions [n_steps, E, N, 4] uint8, one launch. With
 * validate_actions every row is checked, the dead agents' rows included (deaths within the
 * rollout are not known when the check runs).
 */
int macm_tdm_rollout(macm_tdm* w, const void* actions, int32_t n_steps, const macm_tdm_outputs* out, void* stream);

/* The closed loop `step -> bots.combat -> step` in one launch (as macm_world_rollout_bots);
 * actions uint8 [E, N, 4] in/out, out->obs and out->mask must be set. */
int macm_tdm_rollout_bots(macm_tdm* w, uint8_t* actions, int32_t n_steps, const macm_tdm_outputs* out, void* stream);

/* Trajectory forms of the two above (as macm_world_rollout_traj): obs [n_steps, E, N, N-1, 4],
 * mask [n_steps, E, N, N-1], health / alive [n_steps, E, N], done / winner [n_steps, E]; bots:
 * actions [n_steps + 1, E, N, 4]. */
int macm_tdm_rollout_traj(macm_tdm* w, const void* actions, int32_t n_steps, const macm_tdm_outputs* traj,
                          void* stream);
int macm_tdm_rollout_bots_traj(macm_tdm* w, uint8_t* actions, int32_t n_steps, const macm_tdm_outputs* traj,
                               void* stream);

/* TDM.get_obs of the current state without stepping. */
int macm_tdm_observe(macm_tdm* w, const macm_tdm_outputs* out, void* stream);

int macm_tdm_get_state(macm_tdm* w, const macm_tdm_state* dst, void* stream);
int macm_tdm_set_state(macm_tdm* w, const macm_tdm_state* src, void* stream);
int macm_tdm_status(macm_tdm* w, int32_t* status_or, void* stream);

/* out[0] alive agent-steps, out[1] melee attacks, out[2] deaths, out[3] env-steps with done. */
int macm_tdm_counters(macm_tdm* w, int64_t out[4], void* stream);

/* Env-steps taken by the spill step since creation (ABI 6). */
int macm_tdm_spilled(macm_tdm* w, int64_t* env_steps, void* stream);

/* MACM_LAUNCH_* of the next macm_tdm_step / rollout (not the closed loop) (ABI 9). */
int macm_tdm_launch_flags(const macm_tdm* w);

/* Allocates ahead what trajectory rollouts of up to n_steps steps need (the tail observation's pose
 * snapshots, MACM_LAUNCH_TAIL_OBS), so that the rollout itself does not reallocate (a reallocation
 * synchronises its stream); optional (a rollout grows what it needs). Synchronises `stream`. */
int macm_tdm_reserve(macm_tdm* w, int32_t n_steps, void* stream);

/* Test hooks: MACM_DEBUG_FORCE_SPILL, MACM_DEBUG_SPILL_POOL (ABI 6). */
int macm_tdm_set_debug(macm_tdm* w, int32_t flags);

/* ---- scripted actors on the device (test_scripts/bots.py) ------------------
 * Read an observation tensor written by a step and write the next actions, so a
 * closed-loop rollout stays in HBM. Device pointers; asynchronous on `stream`.
 * With float64 obs the decisions equal the reference bots' on the same obs.
 */

/* bots.flock (bots.py:37-61) on Flock obs [rows, obs_dim] (4 polar, 6 cartesian);
 * actions [rows, 3] uint8. rows = E * N. */
int macm_bots_flock(const void* obs, int32_t obs_f64, int32_t obs_dim, int64_t rows, uint8_t* actions,
                    void* stream);

/* bots.combat (bots.py:3-16) on TDM obs [rows, N-1, 4] + mask [rows, N-1];
 * actions [rows, 4] uint8 (rows of dead agents get the idle action). rows = E * N. */
int macm_bots_combat(const void* obs, const uint8_t* mask, int32_t obs_f64, int32_t n_agents, int64_t rows,
                     uint8_t* actions, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MACM_H */
