/*
 * flock_oracle.c — ORACLE / TEST INFRASTRUCTURE ONLY. Never linked into the
 * product (gym-macm_amd/); loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py only.
 *
 * Batched CPU restatement of the reference env layer, gym_macm/envs/mvmnt.py,
 * driving the b2lite world (b2lite.c) exactly the way Flock drives pybox2d:
 *   construction      mvmnt.py:35-79   (RNG order: targets (angle, dist), then
 *                                       agents (x, y, uniform(-1,1)*pi))
 *   step, discrete    mvmnt.py:97-118  (angle set via SetTransform, f64 force math
 *                                       rounded to f32 by ApplyForce)
 *   step, continuous  mvmnt.py:120-129 (float32 arithmetic: gym's Box.contains
 *                                       only admits float32 arrays)
 *   physics           cm_framework.py:172-225 -> b2World.Step(1/hz, 8, 3), ClearForces
 *   rewards           mvmnt.py:160-179 (every agent in world.contacts gets -1)
 *   time / done       mvmnt.py:134-136
 *   obs               mvmnt.py:181-222 (strict '<' nearest neighbour, one wrap)
 * Each env e is the reference env constructed right after random.seed(seed + e).
 * Double math uses glibc libm; numpy's arctan2 can differ from it by 1 ulp (f64),
 * which the tests tolerate (see tests/test_oracle_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/macm.h"
#include "b2lite.h"
#include "pyrandom.h"

#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  b2l_world* w;
  float* targets; /* [T][2] */
  double time_passed;
  int done;
  int step_count;
  pyrandom rng;   /* the env's `random` stream, continued by fo_reset_envs */
} fo_env;

typedef struct fo_batch {
  macm_config cfg;
  int E, N, T, OD;
  int* tidx;
  fo_env* envs;
  float dt;
} fo_batch;

static int obs_dim(const macm_config* c) { return c->coord == MACM_COORD_CARTESIAN ? 6 : 4; }

int fo_obs_dim(const fo_batch* b) { return b->OD; }

static b2l_world* new_world(void) {
  /* FrameworkBase.__init__: b2World(gravity=(0, 0), doSleep=True) (cm_framework.py:161) */
  return b2l_world_new(0.0f, 0.0f, 1);
}

static void body_def(const macm_config* c, b2l_body_def* d, float x, float y, float a) {
  memset(d, 0, sizeof(*d));
  d->x = x;
  d->y = y;
  d->angle = a;
  d->linear_damping = c->linear_damping; /* bodySettings, settings.py:133 */
  d->fixed_rotation = 1;
  d->allow_sleep = 1;
  d->radius = c->radius;
  d->density = c->density;
  d->friction = c->friction;
  d->restitution = 0.0f;
}

static void env_agents(fo_batch* b, fo_env* e) {
  const macm_config* c = &b->cfg;
  pyrandom* r = &e->rng;
  /* mvmnt.py:60-76 */
  for (int i = 0; i < b->N; ++i) {
    double x = c->start_spread * (pyrandom_random(r) - 0.5) + c->start_point[0];
    double y = c->start_spread * (pyrandom_random(r) - 0.5) + c->start_point[1];
    double angle = pyrandom_uniform(r, -1, 1) * M_PI;
    b2l_body_def d;
    body_def(c, &d, (float)x, (float)y, (float)angle);
    b2l_create_body(e->w, &d);
  }
  e->time_passed = 0.0;
  e->done = 0;
  e->step_count = 0;
}

static void env_init(fo_batch* b, fo_env* e, uint64_t seed) {
  const macm_config* c = &b->cfg;
  pyrandom* rp = &e->rng;
  pyrandom_seed(rp, seed);
  pyrandom r = *rp; /* targets drawn from the stream, then agents (env_agents) */
  e->w = new_world();
  e->targets = (float*)malloc(sizeof(float) * 2 * (size_t)b->T);
  /* mvmnt.py:46-52 */
  for (int t = 0; t < b->T; ++t) {
    double rand_angle = 2 * M_PI * pyrandom_random(&r);
    double rand_dist = c->target_mindist + pyrandom_random(&r) * (c->target_maxdist - c->target_mindist);
    e->targets[2 * t + 0] = (float)(rand_dist * cos(rand_angle));
    e->targets[2 * t + 1] = (float)(rand_dist * sin(rand_angle));
  }
  *rp = r;
  env_agents(b, e);
}

/* The working reset (gym_macm/envs/mvmnt.py Flock.reset in this build; the
 * reference's raises at mvmnt.py:227): next agent poses from the env's stream,
 * targets kept, a fresh world. */
void fo_reset_envs(fo_batch* b, const uint8_t* mask) {
  for (int e = 0; e < b->E; ++e) {
    if (mask && !mask[e]) continue;
    fo_env* en = &b->envs[e];
    b2l_world_free(en->w);
    en->w = new_world();
    env_agents(b, en);
  }
}

fo_batch* fo_create(const macm_config* cfg, const int32_t* targets_idx, int n_envs, uint64_t seed,
                    int64_t env_offset) {
  if (!cfg || n_envs <= 0 || cfg->n_agents < 2 || cfg->n_targets < 1) return NULL;
  fo_batch* b = (fo_batch*)calloc(1, sizeof(*b));
  b->cfg = *cfg;
  b->E = n_envs;
  b->N = cfg->n_agents;
  b->T = cfg->n_targets;
  b->OD = obs_dim(cfg);
  b->dt = (float)(1.0 / cfg->hz); /* cm_framework.py:182-185 -> SWIG float32 */
  b->tidx = (int*)calloc((size_t)b->N, sizeof(int));
  for (int i = 0; i < b->N; ++i) b->tidx[i] = targets_idx ? targets_idx[i] : 0;
  b->envs = (fo_env*)calloc((size_t)n_envs, sizeof(fo_env));
  for (int e = 0; e < n_envs; ++e) env_init(b, &b->envs[e], seed + (uint64_t)(env_offset + e));
  return b;
}

void fo_free(fo_batch* b) {
  if (!b) return;
  for (int e = 0; e < b->E; ++e) {
    b2l_world_free(b->envs[e].w);
    free(b->envs[e].targets);
  }
  free(b->envs);
  free(b->tidx);
  free(b);
}

static inline double sgn(double x) { return (x > 0) - (x < 0); }

static inline float distsq(float ax, float ay, float bx, float by) {
  /* b2DistanceSquared(a, b) */
  float cx = ax - bx, cy = ay - by;
  return cx * cx + cy * cy;
}

static void write_node(const macm_config* c, double* o, double r, double t) {
  if (c->coord == MACM_COORD_CARTESIAN) {
    o[0] = r;
    o[1] = cos(t);
    o[2] = sin(t);
  } else {
    o[0] = r;
    o[1] = t;
  }
}

/* Flock.get_obs (mvmnt.py:181-222) for one env */
static void env_obs(const fo_batch* b, const fo_env* e, double* obs, int32_t* nbr) {
  const int N = b->N, OD = b->OD;
  const macm_config* c = &b->cfg;
  float px[4096], py[4096], pa[4096];
  float* X = px;
  float* Y = py;
  float* A = pa;
  float* heap = NULL;
  if (N > 4096) {
    heap = (float*)malloc(sizeof(float) * 3 * (size_t)N);
    X = heap; Y = heap + N; A = heap + 2 * N;
  }
  for (int i = 0; i < N; ++i) {
    float s[7];
    b2l_body_get(e->w, i, s);
    X[i] = s[0]; Y[i] = s[1]; A[i] = s[2];
  }
  for (int i = 0; i < N; ++i) {
    double closest = INFINITY;
    int cj = -1;
    for (int j = 0; j < N; ++j) {
      if (j == i) continue;
      double r = sqrt((double)distsq(X[j], Y[j], X[i], Y[i]));
      if (r < closest) { closest = r; cj = j; }
    }
    float relx = X[cj] - X[i], rely = Y[cj] - Y[i];
    double t = atan2((double)rely, (double)relx) - (double)A[i];
    t = fabs(t) > M_PI ? t - sgn(t) * 2 * M_PI : t;
    double* o = obs + ((size_t)i) * OD;
    write_node(c, o, closest, t);
    if (nbr) nbr[i] = cj;
    const float* tg = e->targets + 2 * b->tidx[i];
    float trx = tg[0] - X[i], try_ = tg[1] - Y[i];
    double r = sqrt((double)distsq(tg[0], tg[1], X[i], Y[i]));
    t = atan2((double)try_, (double)trx) - (double)A[i];
    t = fabs(t) > M_PI ? t - sgn(t) * 2 * M_PI : t;
    write_node(c, o + OD / 2, r, t);
  }
  free(heap);
}

void fo_observe(fo_batch* b, double* obs, int32_t* nbr) {
  for (int e = 0; e < b->E; ++e)
    env_obs(b, &b->envs[e], obs + (size_t)e * b->N * b->OD, nbr ? nbr + (size_t)e * b->N : NULL);
}

static void env_step(fo_batch* b, fo_env* e, const void* actions_env, double* obs, int32_t* nbr,
                     double* reward, uint8_t* collided, uint8_t* done) {
  const macm_config* c = &b->cfg;
  const int N = b->N;
  b2l_world* w = e->w;
  if (c->action_mode == MACM_ACTION_DISCRETE) {
    const uint8_t* act = (const uint8_t*)actions_env;
    for (int i = 0; i < N; ++i) {
      const int a0 = act[3 * i + 0], a1 = act[3 * i + 1], a2 = act[3 * i + 2];
      float s[7];
      b2l_body_get(w, i, s);
      /* agent.body.angle = angle + (a2-1) * rotation_speed * (1/hz)   (:103-104) */
      double ang = (double)s[2] + ((double)(a2 - 1) * c->agent_rotation_speed) * (1 / c->hz);
      b2l_body_set_transform(w, i, s[0], s[1], (float)ang);
      b2l_body_get(w, i, s);
      /* wrap (:105-106) */
      if (fabs((double)s[2]) > M_PI) {
        double na = (double)s[2] - sgn((double)s[2]) * (2 * M_PI);
        b2l_body_set_transform(w, i, s[0], s[1], (float)na);
        b2l_body_get(w, i, s);
      }
      double angle = (double)s[2];
      double cc = ((a0 != 1) && (a1 != 1)) ? 1 / sqrt(2.0) : 1.0; /* :112 */
      double fx = (cos(angle) * (double)(a0 - 1) + cos(angle + M_PI / 2) * (double)(a1 - 1)) * cc * c->agent_force;
      double fy = (sin(angle) * (double)(a0 - 1) + sin(angle + M_PI / 2) * (double)(a1 - 1)) * cc * c->agent_force;
      b2l_body_apply_force(w, i, (float)fx, (float)fy, s[0], s[1], 1); /* :118 */
    }
  } else {
    const float* act = (const float*)actions_env;
    for (int i = 0; i < N; ++i) {
      float x = act[2 * i + 0], y = act[2 * i + 1];
      /* mvmnt.py:122-126 in float32 (numpy float32 scalars) */
      if ((x * x + y * y) > 1.0f) {
        x = sqrtf(x * x / (x * x + y * y));
        y = sqrtf(y * y / (x * x + y * y));
      }
      float fx = x * (float)c->agent_force;
      float fy = y * (float)c->agent_force;
      float s[7];
      b2l_body_get(w, i, s);
      b2l_body_apply_force(w, i, fx, fy, s[0], s[1], 1);
    }
  }
  /* FrameworkBase.Step (cm_framework.py:213-224) */
  b2l_world_set_flags(w, c->warm_starting, 1, 0);
  b2l_world_step(w, b->dt, c->velocity_iterations, c->position_iterations);
  b2l_world_clear_forces(w);
  e->step_count++;

  /* get_rewards (mvmnt.py:160-179) */
  int ncont = b2l_world_contacts(w, NULL, 0);
  int* cl = (int*)malloc(sizeof(int) * 3 * (size_t)(ncont ? ncont : 1));
  b2l_world_contacts(w, cl, ncont);
  uint8_t* hit = collided;
  uint8_t local_hit[4096];
  if (!hit) hit = N <= 4096 ? local_hit : (uint8_t*)malloc((size_t)N);
  memset(hit, 0, (size_t)N);
  for (int k = 0; k < ncont; ++k) { hit[cl[3 * k]] = 1; hit[cl[3 * k + 1]] = 1; }
  free(cl);
  for (int i = 0; i < N; ++i) {
    if (hit[i]) { reward[i] = -1.0; continue; }
    float s[7];
    b2l_body_get(w, i, s);
    const float* tg = e->targets + 2 * b->tidx[i];
    double d = sqrt((double)distsq(tg[0], tg[1], s[0], s[1]));
    if (c->reward_mode == MACM_REWARD_LINEAR) reward[i] = (-d / 35) + 1;
    else reward[i] = (double)(d < c->reward_radius);
  }
  if (!collided && hit != local_hit) free(hit);
  /* time (mvmnt.py:134-136) */
  e->time_passed += (1 / c->hz);
  if (e->time_passed > c->time_limit) e->done = 1;
  if (done) *done = (uint8_t)e->done;
  env_obs(b, e, obs, nbr);
}

void fo_step(fo_batch* b, const void* actions, double* obs, int32_t* nbr, double* reward,
             uint8_t* collided, uint8_t* done, int n_threads) {
  const size_t astride = b->cfg.action_mode == MACM_ACTION_DISCRETE ? (size_t)b->N * 3 : (size_t)b->N * 2 * sizeof(float);
  if (n_threads <= 0) n_threads = 1;
  (void)n_threads;
#pragma omp parallel for num_threads(n_threads) schedule(dynamic, 4)
  for (int e = 0; e < b->E; ++e) {
    env_step(b, &b->envs[e], (const uint8_t*)actions + astride * (size_t)e,
             obs + (size_t)e * b->N * b->OD, nbr ? nbr + (size_t)e * b->N : NULL,
             reward + (size_t)e * b->N, collided ? collided + (size_t)e * b->N : NULL,
             done ? done + e : NULL);
  }
}

/* All contacts of env e in world-list order: [a, b, touching]. */
int fo_contacts(fo_batch* b, int e, int* out3, int cap) { return b2l_world_contacts(b->envs[e].w, out3, cap); }

static int fat_overlap(const float* a, const float* b) {
  float d1x = b[0] - a[2], d1y = b[1] - a[3];
  float d2x = a[0] - b[2], d2y = a[1] - b[3];
  if (d1x > 0.0f || d1y > 0.0f) return 0;
  if (d2x > 0.0f || d2y > 0.0f) return 0;
  return 1;
}

/*
 * Export one world's bodies and contacts in the product's macm_state layout
 * (include/macm.h), env slot e. The ordered contact list is the world list
 * filtered to the pairs whose CURRENT fat AABBs overlap (the contacts that survive
 * the next Collide), with the warm-start impulses of contacts that carry a
 * manifold point. Shared with tdm_oracle.c.
 */
void fo_export_world(b2l_world* w, int N, size_t e, float* pos, float* vel, float* angle, float* fat,
                     float* sleep, int32_t* contact_count, uint32_t* contact_ab, float* contact_imp,
                     int max_contacts) {
  for (int i = 0; i < N; ++i) {
    float s[7], f[4];
    b2l_body_get(w, i, s);
    b2l_body_get_fat(w, i, f);
    size_t k = e * N + i;
    if (pos) { pos[2 * k] = s[0]; pos[2 * k + 1] = s[1]; }
    if (vel) { vel[2 * k] = s[3]; vel[2 * k + 1] = s[4]; }
    if (angle) angle[k] = s[2];
    if (sleep) sleep[k] = s[5];
    if (fat) memcpy(fat + 4 * k, f, sizeof(f));
  }
  if (!contact_count) return;
  b2l_world_flush_new_contacts(w);
  int n = b2l_world_contacts(w, NULL, 0);
  int* cl = (int*)malloc(sizeof(int) * 3 * (size_t)(n ? n : 1));
  float* im = (float*)malloc(sizeof(float) * 3 * (size_t)(n ? n : 1));
  b2l_world_contacts(w, cl, n);
  b2l_world_contact_impulses(w, im, n);
  int m = 0;
  for (int k = 0; k < n; ++k) {
    float fa[4], fb[4];
    b2l_body_get_fat(w, cl[3 * k], fa);
    b2l_body_get_fat(w, cl[3 * k + 1], fb);
    if (!fat_overlap(fa, fb)) continue;
    if (m < max_contacts) {
      size_t o = e * max_contacts + m;
      contact_ab[o] = (uint32_t)cl[3 * k] | ((uint32_t)cl[3 * k + 1] << 16);
      int pc = (int)im[3 * k + 2];
      contact_imp[2 * o] = pc > 0 ? im[3 * k] : 0.0f;
      contact_imp[2 * o + 1] = pc > 0 ? im[3 * k + 1] : 0.0f;
    }
    ++m;
  }
  contact_count[e] = m;
  free(cl);
  free(im);
}

/* Inverse of fo_export_world: body states, then the ordered list (see b2l_world_load_contacts). */
void fo_import_world(b2l_world* w, int N, size_t e, const float* pos, const float* vel, const float* angle,
                     const float* fat, const float* sleep, const int32_t* contact_count,
                     const uint32_t* contact_ab, const float* contact_imp, int max_contacts) {
  for (int i = 0; i < N; ++i) {
    size_t k = e * N + i;
    b2l_body_set_state(w, i, pos[2 * k], pos[2 * k + 1], angle[k], vel[2 * k], vel[2 * k + 1], sleep[k],
                       fat + 4 * k);
  }
  int n = contact_count[e];
  int* ab = (int*)malloc(sizeof(int) * 2 * (size_t)(n ? n : 1));
  int* pc = (int*)malloc(sizeof(int) * (size_t)(n ? n : 1));
  for (int k = 0; k < n; ++k) {
    uint32_t v = contact_ab[e * max_contacts + k];
    ab[2 * k] = (int)(v & 0xffffu);
    ab[2 * k + 1] = (int)(v >> 16);
    const float* im = contact_imp + 2 * (e * max_contacts + k);
    pc[k] = (im[0] != 0.0f || im[1] != 0.0f) ? 1 : 0;
  }
  b2l_world_load_contacts(w, n, ab, contact_imp + 2 * e * max_contacts, pc);
  free(ab);
  free(pc);
}

void fo_get_state(fo_batch* b, float* pos, float* vel, float* angle, float* fat, float* sleep,
                  float* targets, int32_t* contact_count, uint32_t* contact_ab, float* contact_imp,
                  int max_contacts, int32_t* step_count, double* time_passed) {
  for (int e = 0; e < b->E; ++e) {
    fo_env* en = &b->envs[e];
    fo_export_world(en->w, b->N, (size_t)e, pos, vel, angle, fat, sleep, contact_count, contact_ab, contact_imp,
                    max_contacts);
    if (targets) memcpy(targets + (size_t)e * 2 * b->T, en->targets, sizeof(float) * 2 * (size_t)b->T);
    if (step_count) step_count[e] = en->step_count;
    if (time_passed) time_passed[e] = en->time_passed;
  }
}

void fo_set_state(fo_batch* b, const float* pos, const float* vel, const float* angle,
                  const float* fat, const float* sleep, const float* targets,
                  const int32_t* contact_count, const uint32_t* contact_ab, const float* contact_imp,
                  int max_contacts, const int32_t* step_count, const double* time_passed) {
  for (int e = 0; e < b->E; ++e) {
    fo_env* en = &b->envs[e];
    fo_import_world(en->w, b->N, (size_t)e, pos, vel, angle, fat, sleep, contact_count, contact_ab, contact_imp,
                    max_contacts);
    memcpy(en->targets, targets + (size_t)e * 2 * b->T, sizeof(float) * 2 * (size_t)b->T);
    en->step_count = step_count[e];
    en->time_passed = time_passed[e];
    en->done = en->time_passed > b->cfg.time_limit;
    b2l_world_set_solver_state(en->w, en->step_count > 0 ? 1.0f / b->dt : 0.0f, 0);
  }
}

/* ---- low-level world API re-exported for the Box2D facade used to run the
 *      reference's own env code when generating golden vectors ------------ */
b2l_world* fo_world_new(void) { return new_world(); }
