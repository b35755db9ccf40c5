/*
 * tdm_oracle.c — ORACLE / TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench
 * cpu_baseline). Batched CPU restatement of the reference TDM env,
 * gym_macm/envs/combat.py:57-227, over the b2lite world.
 *
 * The reference cannot construct or step TDM as shipped. The four missing names
 * are supplied from combatSettings (settings.py:149-177) exactly as
 * tests/golden/make_golden.py patches them at run time:
 *   combatSettings (combat.py:65, import missing at :8),
 *   self.cooldown_atk, self.cooldown_mov_penalty (:150-151), self.time_limit (:173).
 * Everything else is literal (cfg->fresh_raycast = cfg->decay_mov_penalty = 0),
 * including two reference behaviours the config can switch off:
 *   * ONE shared RayCastClosestCallback whose `hit`/`fixture` are never reset
 *     (cm_framework.py:62-65,76): once anything has been hit, every later attack
 *     damages the last-hit fixture's body even when its own ray misses;
 *   * cooldown_mov_penalty is set on attack and never decremented (:151,:155), so
 *     an agent that has attacked keeps force 20 * (1 - 0.2) for the episode.
 * Deaths: body.active = False (:162) destroys the proxy and the body's contacts.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/macm.h"
#include "b2lite.h"
#include "pyrandom.h"

typedef struct {
  b2l_world* w;
  double* health;
  double* cd_atk;
  double* cd_mov;
  uint8_t* alive;
  int n_alive[4];
  int listener_hit;      /* RayCastClosestCallback.hit, never reset        */
  int listener_body;     /* body of RayCastClosestCallback.fixture (or -1) */
  double time_passed;
  int done, winner;
  int step_count;
  pyrandom rng;          /* the env's `random` stream, continued by to_reset_envs */
} to_env;

typedef struct to_batch {
  macm_tdm_config cfg;
  int E, N;
  int* team;
  to_env* envs;
  float dt;
} to_batch;

static inline double sgn(double x) { return (x > 0) - (x < 0); }
static inline double wrap(double t) { return fabs(t) > M_PI ? t - sgn(t) * 2 * M_PI : t; }

/* combat.py:78-101: a new world, bodies at poses drawn from the env's stream. */
static void env_spawn(const to_batch* b, to_env* en) {
  const macm_tdm_config* cfg = &b->cfg;
  const int N = b->N;
  en->w = b2l_world_new(0.0f, 0.0f, 1);
  for (int i = 0; i < N; ++i) { /* combat.py:80-95 */
    double x = pyrandom_random(&en->rng) * (b->team[i] + cfg->world_width / 2);
    double y = pyrandom_random(&en->rng) * cfg->world_height;
    double angle = pyrandom_uniform(&en->rng, -1, 1) * M_PI;
    b2l_body_def d;
    memset(&d, 0, sizeof(d));
    d.x = (float)x; d.y = (float)y; d.angle = (float)angle;
    d.linear_damping = cfg->linear_damping; d.fixed_rotation = 1; d.allow_sleep = 1;
    d.radius = cfg->radius; d.density = cfg->density; d.friction = cfg->friction;
    b2l_create_body(en->w, &d);
    en->health[i] = cfg->init_health;
    en->cd_atk[i] = 0.0;
    en->cd_mov[i] = 0.0;
    en->alive[i] = 1;
  }
  for (int t = 0; t < cfg->n_teams; ++t) en->n_alive[t] = cfg->team_size[t];
  en->listener_hit = 0;
  en->listener_body = -1;
  en->winner = -1;
  en->done = 0;
  en->time_passed = 0.0;
  en->step_count = 0;
}

to_batch* to_create(const macm_tdm_config* cfg, int n_envs, uint64_t seed, int64_t env_offset) {
  if (!cfg || n_envs <= 0 || cfg->n_teams < 1 || cfg->n_teams > 4) return NULL;
  to_batch* b = (to_batch*)calloc(1, sizeof(*b));
  b->cfg = *cfg;
  b->E = n_envs;
  int N = 0;
  for (int t = 0; t < cfg->n_teams; ++t) N += cfg->team_size[t];
  b->N = N;
  b->dt = (float)(1.0 / cfg->hz);
  b->team = (int*)calloc((size_t)N, sizeof(int));
  for (int t = 0, i = 0; t < cfg->n_teams; ++t)
    for (int j = 0; j < cfg->team_size[t]; ++j) b->team[i++] = t;
  b->envs = (to_env*)calloc((size_t)n_envs, sizeof(to_env));
  for (int e = 0; e < n_envs; ++e) {
    to_env* en = &b->envs[e];
    pyrandom_seed(&en->rng, seed + (uint64_t)(env_offset + e));
    en->health = (double*)calloc((size_t)N, sizeof(double));
    en->cd_atk = (double*)calloc((size_t)N, sizeof(double));
    en->cd_mov = (double*)calloc((size_t)N, sizeof(double));
    en->alive = (uint8_t*)calloc((size_t)N, 1);
    env_spawn(b, en);
  }
  return b;
}

/* This build's working reset (the reference's, combat.py:234-245, leaves dead
 * bodies inactive): next spawn poses from the env's stream, a fresh world, every
 * agent alive with init_health and zero cooldowns, a fresh listener. */
void to_reset_envs(to_batch* b, const uint8_t* mask) {
  for (int e = 0; e < b->E; ++e) {
    if (mask && !mask[e]) continue;
    to_env* en = &b->envs[e];
    b2l_world_free(en->w);
    env_spawn(b, en);
  }
}

void to_free(to_batch* b) {
  if (!b) return;
  for (int e = 0; e < b->E; ++e) {
    to_env* en = &b->envs[e];
    b2l_world_free(en->w);
    free(en->health); free(en->cd_atk); free(en->cd_mov); free(en->alive);
  }
  free(b->envs);
  free(b->team);
  free(b);
}

int to_n_agents(const to_batch* b) { return b->N; }

/* TDM.get_obs (combat.py:206-227) as fixed slots: agent i, slot k -> other agent
 * j = k < i ? k : k + 1; (r, t, p, is_ally), mask 1 iff i and j are alive. */
static void env_obs(const to_batch* b, const to_env* en, double* obs, uint8_t* mask) {
  const int N = b->N;
  float s[7];
  float* X = (float*)malloc(sizeof(float) * 3 * (size_t)N); /* any team sizes (combat.py:82-83) */
  float* Y = X + N;
  float* A = Y + N;
  for (int i = 0; i < N; ++i) {
    b2l_body_get(en->w, i, s);
    X[i] = s[0]; Y[i] = s[1]; A[i] = s[2];
  }
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < N - 1; ++k) {
      const int j = k < i ? k : k + 1;
      double* o = obs + ((size_t)i * (N - 1) + k) * 4;
      uint8_t m = en->alive[i] && en->alive[j];
      if (mask) mask[(size_t)i * (N - 1) + k] = m;
      if (!m) { o[0] = o[1] = o[2] = o[3] = 0.0; continue; }
      float rx = X[j] - X[i], ry = Y[j] - Y[i];
      float d2 = rx * rx + ry * ry; /* b2DistanceSquared(other, agent) */
      o[0] = sqrt((double)d2);
      o[1] = wrap(atan2((double)ry, (double)rx) - (double)A[i]);
      o[2] = wrap((double)A[j] - (double)A[i]);
      o[3] = (double)(b->team[i] == b->team[j]);
    }
  free(X);
}

void to_observe(to_batch* b, double* obs, uint8_t* mask) {
  const size_t per = (size_t)b->N * (b->N - 1);
  for (int e = 0; e < b->E; ++e) env_obs(b, &b->envs[e], obs + (size_t)e * per * 4, mask ? mask + e * per : NULL);
}

static void env_step(to_batch* b, to_env* en, const uint8_t* act, double* obs, uint8_t* mask) {
  const macm_tdm_config* c = &b->cfg;
  const int N = b->N;
  b2l_world* w = en->w;
  for (int i = 0; i < N; ++i) { /* combat.py:121-155 */
    if (!en->alive[i]) continue;
    const int a0 = act[4 * i], a1 = act[4 * i + 1], a2 = act[4 * i + 2], a3 = act[4 * i + 3];
    float s[7];
    b2l_body_get(w, i, s);
    double ang = (double)s[2] + ((double)(a2 - 1) * c->agent_rotation_speed) * (1 / c->hz);
    b2l_body_set_transform(w, i, s[0], s[1], (float)ang);
    b2l_body_get(w, i, s);
    if (fabs((double)s[2]) > M_PI) {
      b2l_body_set_transform(w, i, s[0], s[1], (float)((double)s[2] - sgn((double)s[2]) * (2 * M_PI)));
      b2l_body_get(w, i, s);
    }
    const double angle = (double)s[2];
    const double cc = ((a0 != 1) && (a1 != 1)) ? 1 / sqrt(2.0) : 1.0;
    const double force = c->agent_force * (1 - c->percent_mov_penalty * (double)(en->cd_mov[i] > 0)); /* :46-49 */
    const double fx = (cos(angle) * (double)(a0 - 1) + cos(angle + M_PI / 2) * (double)(a1 - 1)) * cc * force;
    const double fy = (sin(angle) * (double)(a0 - 1) + sin(angle + M_PI / 2) * (double)(a1 - 1)) * cc * force;
    b2l_body_apply_force(w, i, (float)fx, (float)fy, s[0], s[1], 1);
    if (en->cd_atk[i] <= 0) {
      if (a3) {
        /* point2 = point1 + (range*cos(angle), range*sin(angle)): b2Vec2 + tuple
         * -> float32 vector add of the float32-converted tuple */
        const double ang2 = (double)s[2];
        const float dx = (float)(c->melee_range * cos(ang2)), dy = (float)(c->melee_range * sin(ang2));
        const float x2 = s[0] + dx, y2 = s[1] + dy;
        const int hit = b2l_world_raycast(w, s[0], s[1], x2, y2, NULL);
        en->cd_atk[i] = c->cooldown_atk;
        en->cd_mov[i] = c->cooldown_mov_penalty;
        if (c->fresh_raycast) {
          if (hit >= 0) en->health[hit] -= c->melee_dmg;
        } else {
          if (hit >= 0) { en->listener_hit = 1; en->listener_body = hit; }
          if (en->listener_hit) en->health[en->listener_body] -= c->melee_dmg;
        }
      }
    } else {
      en->cd_atk[i] -= (1 / c->hz);
      if (c->decay_mov_penalty) en->cd_mov[i] -= (1 / c->hz);
    }
  }
  for (int i = 0; i < N; ++i) { /* deaths, combat.py:157-165 */
    if (!en->alive[i]) continue;
    if (en->health[i] <= 0) {
      en->alive[i] = 0;
      b2l_body_set_active(w, i, 0);
      en->n_alive[b->team[i]] -= 1;
    }
  }
  b2l_world_set_flags(w, c->warm_starting, 1, 0);
  b2l_world_step(w, b->dt, c->velocity_iterations, c->position_iterations);
  b2l_world_clear_forces(w);
  en->step_count++;
  env_obs(b, en, obs, mask);
  en->time_passed += (1 / c->hz); /* :171-182 */
  int alive_teams = 0, last = -1;
  for (int t = 0; t < c->n_teams; ++t)
    if (en->n_alive[t] != 0) { ++alive_teams; last = t; }
  if (en->time_passed > c->time_limit) en->done = 1;
  if (alive_teams == 1) { en->done = 1; en->winner = last; }
  if (alive_teams == 0) en->done = 1;
}

void to_step(to_batch* b, const uint8_t* actions, double* obs, uint8_t* mask, double* health, uint8_t* alive,
             uint8_t* done, int32_t* winner, int n_threads) {
  const int N = b->N;
  const size_t per = (size_t)N * (N - 1);
  if (n_threads <= 0) n_threads = 1;
  (void)n_threads;
#pragma omp parallel for num_threads(n_threads) schedule(dynamic, 4)
  for (int e = 0; e < b->E; ++e) {
    to_env* en = &b->envs[e];
    env_step(b, en, actions + (size_t)e * N * 4, obs + (size_t)e * per * 4, mask ? mask + e * per : NULL);
    if (health) memcpy(health + (size_t)e * N, en->health, sizeof(double) * N);
    if (alive) memcpy(alive + (size_t)e * N, en->alive, (size_t)N);
    if (done) done[e] = (uint8_t)en->done;
    if (winner) winner[e] = en->winner;
  }
}

/* Per-env TDM extras for parity: cd_atk, cd_mov [E,N] f64, listener [E,2] (hit, body). */
void to_get_extras(const to_batch* b, double* cd_atk, double* cd_mov, int32_t* listener) {
  for (int e = 0; e < b->E; ++e) {
    const to_env* en = &b->envs[e];
    memcpy(cd_atk + (size_t)e * b->N, en->cd_atk, sizeof(double) * b->N);
    memcpy(cd_mov + (size_t)e * b->N, en->cd_mov, sizeof(double) * b->N);
    listener[2 * e] = en->listener_hit;
    listener[2 * e + 1] = en->listener_body;
  }
}

b2l_world* to_world(to_batch* b, int e) { return b->envs[e].w; }

void fo_export_world(b2l_world* w, int N, size_t e, float* pos, float* vel, float* angle, float* fat,
                     float* sleep, int32_t* contact_count, uint32_t* contact_ab, float* contact_imp,
                     int max_contacts);
void fo_import_world(b2l_world* w, int N, size_t e, const float* pos, const float* vel, const float* angle,
                     const float* fat, const float* sleep, const int32_t* contact_count,
                     const uint32_t* contact_ab, const float* contact_imp, int max_contacts);

/* Export in the product's macm_tdm_state layout (include/macm.h); NULL = skip. */
void to_get_state(to_batch* b, float* pos, float* vel, float* angle, float* fat, float* sleep, double* health,
                  double* cd_atk, double* cd_mov, uint8_t* alive, int32_t* listener, int32_t* contact_count,
                  uint32_t* contact_ab, float* contact_imp, int max_contacts, int32_t* step_count,
                  double* time_passed, uint8_t* done, int32_t* winner) {
  const int N = b->N;
  for (int e = 0; e < b->E; ++e) {
    to_env* en = &b->envs[e];
    fo_export_world(en->w, N, (size_t)e, pos, vel, angle, fat, sleep, contact_count, contact_ab, contact_imp,
                    max_contacts);
    const size_t o = (size_t)e * N;
    if (health) memcpy(health + o, en->health, sizeof(double) * N);
    if (cd_atk) memcpy(cd_atk + o, en->cd_atk, sizeof(double) * N);
    if (cd_mov) memcpy(cd_mov + o, en->cd_mov, sizeof(double) * N);
    if (alive) memcpy(alive + o, en->alive, (size_t)N);
    if (listener) { listener[2 * e] = en->listener_hit; listener[2 * e + 1] = en->listener_body; }
    if (step_count) step_count[e] = en->step_count;
    if (time_passed) time_passed[e] = en->time_passed;
    if (done) done[e] = (uint8_t)en->done;
    if (winner) winner[e] = en->winner;
  }
}

/* Import a macm_tdm_state (all pointers required). Bodies marked dead are
 * deactivated (their contacts destroyed) before the contact list is loaded; a
 * dead body cannot be revived. */
void to_set_state(to_batch* b, const float* pos, const float* vel, const float* angle, const float* fat,
                  const float* sleep, const double* health, const double* cd_atk, const double* cd_mov,
                  const uint8_t* alive, const int32_t* listener, const int32_t* contact_count,
                  const uint32_t* contact_ab, const float* contact_imp, int max_contacts, const int32_t* step_count,
                  const double* time_passed, const uint8_t* done, const int32_t* winner) {
  const int N = b->N;
  for (int e = 0; e < b->E; ++e) {
    to_env* en = &b->envs[e];
    const size_t o = (size_t)e * N;
    for (int t = 0; t < b->cfg.n_teams; ++t) en->n_alive[t] = 0;
    for (int i = 0; i < N; ++i) {
      if (!alive[o + i] && en->alive[i]) b2l_body_set_active(en->w, i, 0);
      en->alive[i] = alive[o + i] ? 1 : 0;
      if (en->alive[i]) en->n_alive[b->team[i]]++;
    }
    fo_import_world(en->w, N, (size_t)e, pos, vel, angle, fat, sleep, contact_count, contact_ab, contact_imp,
                    max_contacts);
    memcpy(en->health, health + o, sizeof(double) * N);
    memcpy(en->cd_atk, cd_atk + o, sizeof(double) * N);
    memcpy(en->cd_mov, cd_mov + o, sizeof(double) * N);
    en->listener_hit = listener[2 * e];
    en->listener_body = listener[2 * e + 1];
    en->step_count = step_count[e];
    en->time_passed = time_passed[e];
    en->done = done[e];
    en->winner = winner[e];
    b2l_world_set_solver_state(en->w, en->step_count > 0 ? 1.0f / b->dt : 0.0f, 0);
  }
}
