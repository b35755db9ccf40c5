/*
 * b2lite.h — ORACLE / TEST INFRASTRUCTURE ONLY. Not part of the product path.
 *
 * CPU restatement of the Box2D 2.3.x subset that gym-macm's Flock env exercises
 * through pybox2d (reference call sites: gym_macm/cm_framework.py:161,222-224;
 * gym_macm/envs/mvmnt.py:70-75,103-106,118,129,162-164,170,193,210).
 *
 * Box2D itself is a third-party dependency that is NOT present under
 * /root/reference (setup.py:5 does not even declare it; pybox2d 2.3.x wheels
 * wrap Box2D ~2.3.2, version unpinned). This file restates its published
 * algorithm for: dynamic circle bodies with one fixture, fixedRotation, linear
 * damping, sleeping, the dynamic-tree broad phase's fat-AABB/move-buffer/pair
 * semantics (queried by brute force; the query SET is identical), the contact
 * manager's linked world/edge lists, island DFS, and the sequential-impulse
 * contact solver with warm starting. Dynamics fidelity vs real Box2D is
 * therefore "parity unpinned" (no reference test or fixture covers it); it is
 * pinned by analytic known-answer tests in tests/test_oracle_physics.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code.
 */
#ifndef B2LITE_H
#define B2LITE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct b2l_world b2l_world;

typedef struct b2l_body_def {
  float x, y, angle;
  float linear_damping;
  int fixed_rotation;
  int allow_sleep;
  /* one circle fixture at the body origin */
  float radius, density, friction, restitution;
} b2l_body_def;

b2l_world* b2l_world_new(float gx, float gy, int do_sleep);
void b2l_world_free(b2l_world* w);
void b2l_world_set_flags(b2l_world* w, int warm_starting, int continuous, int sub_stepping);

/* b2World::CreateBody + b2Body::CreateFixture(circle). Returns body id (creation index). */
int b2l_create_body(b2l_world* w, const b2l_body_def* def);
int b2l_body_count(const b2l_world* w);

/* Getters: out = {x, y, angle, vx, vy, sleep_time, awake} */
void b2l_body_get(const b2l_world* w, int id, float* out7);
void b2l_body_get_fat(const b2l_world* w, int id, float* out4);
/* b2Body::SetTransform (pybox2d `body.angle = a` calls SetTransform(position, a)). */
void b2l_body_set_transform(b2l_world* w, int id, float x, float y, float angle);
/* b2Body::ApplyForce(force, point, wake). */
void b2l_body_apply_force(b2l_world* w, int id, float fx, float fy, float px, float py, int wake);

/* b2World::Step(dt, velocityIterations, positionIterations) and ClearForces. */
void b2l_world_step(b2l_world* w, float dt, int vel_iters, int pos_iters);
void b2l_world_clear_forces(b2l_world* w);

/* world.contacts in world-list order. out: [a, b, touching] per contact (a = fixtureA body).
 * Returns the number of contacts (writes at most cap). */
int b2l_world_contacts(const b2l_world* w, int* out3, int cap);
/* Per touching-or-not contact impulses in world-list order: [normal, tangent, pointCount]. */
int b2l_world_contact_impulses(const b2l_world* w, float* out3, int cap);

/* Rebuild the contact lists from an ordered list (world-list order, head first) of
 * pairs with warm-start impulses; pairs with point_count 0 carry no impulse.
 * Used to inject a state exported by the HIP path. */
void b2l_world_load_contacts(b2l_world* w, int n, const int* ab, const float* imp,
                             const int* point_count);
/* Direct state injection for parity tests. */
void b2l_body_set_state(b2l_world* w, int id, float x, float y, float angle, float vx, float vy,
                        float sleep_time, const float* fat4);
/* Perform the deferred first FindNewContacts now (no-op once stepped). */
void b2l_world_flush_new_contacts(b2l_world* w);
/* b2Body::SetActive(false) (destroys the proxy and every attached contact). */
void b2l_body_set_active(b2l_world* w, int id, int flag);
int b2l_body_active(const b2l_world* w, int id);
/* b2World::RayCast(closest-hit callback); returns the hit body or -1. */
int b2l_world_raycast(const b2l_world* w, float x1, float y1, float x2, float y2, float* fraction_out);
/* World-level solver state: inv_dt0 and the "new fixture" flag. */
void b2l_world_set_solver_state(b2l_world* w, float inv_dt0, int new_fixture);

#ifdef __cplusplus
}
#endif
#endif
