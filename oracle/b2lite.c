/*
 * b2lite.c — ORACLE / TEST INFRASTRUCTURE ONLY (see b2lite.h).
 *
 * Restatement of Box2D 2.3.x [EXT-B2D] semantics used by the reference through
 * pybox2d. Section markers name the Box2D routine each block restates; the
 * reference call site that reaches it is given where there is one.
 *
 * Build with -ffp-contract=off and no -ffast-math: Box2D's x86-64 builds use
 * SSE2 scalar float arithmetic with no FMA, and every expression below keeps
 * Box2D's operand order so the float rounding sequence is the same.
 */
#include "b2lite.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- b2Settings.h constants ------------------------------------------- */
#define B2_PI 3.14159265359f
#define B2_EPS FLT_EPSILON
#define B2_LINEAR_SLOP 0.005f
#define B2_AABB_EXTENSION 0.1f
#define B2_AABB_MULTIPLIER 2.0f
#define B2_MAX_TRANSLATION 2.0f
#define B2_MAX_TRANSLATION_SQ (B2_MAX_TRANSLATION * B2_MAX_TRANSLATION)
#define B2_MAX_ROTATION (0.5f * B2_PI)
#define B2_MAX_ROTATION_SQ (B2_MAX_ROTATION * B2_MAX_ROTATION)
#define B2_BAUMGARTE 0.2f
#define B2_MAX_LINEAR_CORRECTION 0.2f
#define B2_VELOCITY_THRESHOLD 1.0f
#define B2_TIME_TO_SLEEP 0.5f
#define B2_LINEAR_SLEEP_TOL 0.01f
#define B2_ANGULAR_SLEEP_TOL (2.0f / 180.0f * B2_PI)

typedef struct { float x, y; } v2;
typedef struct { v2 lo, hi; } aabb;
typedef struct { float s, c; } rot;
typedef struct { v2 p; rot q; } xform;

static inline v2 V(float x, float y) { v2 r = {x, y}; return r; }
static inline v2 vadd(v2 a, v2 b) { return V(a.x + b.x, a.y + b.y); }
static inline v2 vsub(v2 a, v2 b) { return V(a.x - b.x, a.y - b.y); }
static inline v2 vscale(float s, v2 a) { return V(s * a.x, s * a.y); }
static inline float vdot(v2 a, v2 b) { return a.x * b.x + a.y * b.y; }
static inline float vcross(v2 a, v2 b) { return a.x * b.y - a.y * b.x; }
static inline v2 vcross_vs(v2 a, float s) { return V(s * a.y, -s * a.x); }
static inline v2 vcross_sv(float s, v2 a) { return V(-s * a.y, s * a.x); }
static inline float fminb(float a, float b) { return a < b ? a : b; } /* b2Min */
static inline float fmaxb(float a, float b) { return a > b ? a : b; } /* b2Max */
static inline float fclampb(float a, float lo, float hi) { return fmaxb(lo, fminb(a, hi)); }
static inline v2 vmin(v2 a, v2 b) { return V(fminb(a.x, b.x), fminb(a.y, b.y)); }
static inline v2 vmax(v2 a, v2 b) { return V(fmaxb(a.x, b.x), fmaxb(a.y, b.y)); }
static inline float vlen(v2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
static inline float vdist2(v2 a, v2 b) { v2 c = vsub(a, b); return vdot(c, c); } /* b2DistanceSquared */
/* b2Vec2::Normalize */
static inline float vnormalize(v2* a) {
  float len = vlen(*a);
  if (len < B2_EPS) return 0.0f;
  float inv = 1.0f / len;
  a->x *= inv;
  a->y *= inv;
  return len;
}
static inline rot rot_set(float angle) { rot q; q.s = sinf(angle); q.c = cosf(angle); return q; }
static inline v2 rot_mul(rot q, v2 v) { return V(q.c * v.x - q.s * v.y, q.s * v.x + q.c * v.y); }
static inline v2 xf_mul(xform t, v2 v) {
  float x = (t.q.c * v.x - t.q.s * v.y) + t.p.x;
  float y = (t.q.s * v.x + t.q.c * v.y) + t.p.y;
  return V(x, y);
}
/* b2TestOverlap(a, b) */
static inline int aabb_overlap(aabb a, aabb b) {
  v2 d1 = vsub(b.lo, a.hi), d2 = vsub(a.lo, b.hi);
  if (d1.x > 0.0f || d1.y > 0.0f) return 0;
  if (d2.x > 0.0f || d2.y > 0.0f) return 0;
  return 1;
}
/* b2AABB::Contains */
static inline int aabb_contains(aabb outer, aabb in) {
  int r = 1;
  r = r && outer.lo.x <= in.lo.x;
  r = r && outer.lo.y <= in.lo.y;
  r = r && in.hi.x <= outer.hi.x;
  r = r && in.hi.y <= outer.hi.y;
  return r;
}

/* ---- bodies ------------------------------------------------------------- */
enum { BF_ISLAND = 1, BF_AWAKE = 2, BF_AUTOSLEEP = 4, BF_FIXEDROT = 16, BF_ACTIVE = 32 };

typedef struct {
  xform xf;          /* m_xf */
  v2 local_center;   /* m_sweep.localCenter */
  v2 c0, c;          /* m_sweep.c0, c */
  float a0, a;       /* m_sweep.a0, a */
  v2 v; float w;
  v2 force; float torque;
  float mass, inv_mass, I, inv_I;
  float lin_damp, ang_damp, gravity_scale;
  float sleep_time;
  int flags;
  int island_index;
  int contact_list;  /* head edge id (contact*2 + side) or -1 */
  int prev, next;    /* world body list */
  /* single circle fixture + its one proxy */
  v2 shape_p;        /* circle m_p (local origin) */
  float radius, density, friction, restitution;
  aabb proxy_aabb;   /* b2FixtureProxy::aabb */
  int proxy_id;
} body;

/* ---- contacts ----------------------------------------------------------- */
enum { CF_ISLAND = 1, CF_TOUCHING = 2, CF_ENABLED = 4, CF_FILTER = 8, CF_TOI = 32 };

typedef struct {
  int flags;
  int fa, fb;              /* body ids of fixtureA / fixtureB */
  int prev, next;          /* world contact list */
  int eprev[2], enext[2];  /* edge lists: side 0 = m_nodeA (on fa), side 1 = m_nodeB (on fb) */
  float friction, restitution, tangent_speed;
  /* b2Manifold, circle type: at most one point, local points at shape origins */
  int point_count;
  float normal_impulse, tangent_impulse;
  int alive;
  int next_free;
} contact;

struct b2l_world {
  v2 gravity;
  int allow_sleep, warm_starting, continuous, sub_stepping;
  int new_fixture, step_complete;
  float inv_dt0;

  body* bodies; int nb, bcap;
  int body_list;

  contact* contacts; int ccap; int free_head; int contact_list; int contact_count;

  /* broad phase: fat AABB per proxy (proxy id == body id, see create_body) */
  aabb* fat; int* move_buf; int move_count, move_cap;
  int* pair_buf; int pair_count, pair_cap;

  /* island scratch */
  int* isl_bodies; int* isl_contacts; int* stack;
};

static void* xrealloc(void* p, size_t n) {
  void* q = realloc(p, n);
  if (!q && n) abort();
  return q;
}

b2l_world* b2l_world_new(float gx, float gy, int do_sleep) {
  b2l_world* w = (b2l_world*)calloc(1, sizeof(*w));
  w->gravity = V(gx, gy);
  w->allow_sleep = do_sleep;
  w->warm_starting = 1;
  w->continuous = 1;
  w->sub_stepping = 0;
  w->step_complete = 1;
  w->inv_dt0 = 0.0f;
  w->body_list = -1;
  w->contact_list = -1;
  w->free_head = -1;
  return w;
}

void b2l_world_free(b2l_world* w) {
  if (!w) return;
  free(w->bodies); free(w->contacts); free(w->fat); free(w->move_buf); free(w->pair_buf);
  free(w->isl_bodies); free(w->isl_contacts); free(w->stack);
  free(w);
}

void b2l_world_set_flags(b2l_world* w, int warm, int cont, int sub) {
  w->warm_starting = warm; w->continuous = cont; w->sub_stepping = sub;
}

int b2l_body_count(const b2l_world* w) { return w->nb; }

/* b2BroadPhase::BufferMove */
static void buffer_move(b2l_world* w, int proxy) {
  if (w->move_count == w->move_cap) {
    w->move_cap = w->move_cap ? 2 * w->move_cap : 16;
    w->move_buf = (int*)xrealloc(w->move_buf, sizeof(int) * w->move_cap);
  }
  w->move_buf[w->move_count++] = proxy;
}

/* b2CircleShape::ComputeAABB */
static aabb circle_aabb(const body* b, xform xf) {
  v2 p = vadd(xf.p, rot_mul(xf.q, b->shape_p));
  aabb r;
  r.lo = V(p.x - b->radius, p.y - b->radius);
  r.hi = V(p.x + b->radius, p.y + b->radius);
  return r;
}

/* b2Body::ResetMassData for one circle fixture */
static void reset_mass_data(body* b) {
  b->mass = 0.0f; b->inv_mass = 0.0f; b->I = 0.0f; b->inv_I = 0.0f;
  b->local_center = V(0.0f, 0.0f);
  v2 lc = V(0.0f, 0.0f);
  if (b->density != 0.0f) {
    /* b2CircleShape::ComputeMass */
    float mass = b->density * B2_PI * b->radius * b->radius;
    v2 center = b->shape_p;
    float I = mass * (0.5f * b->radius * b->radius + vdot(b->shape_p, b->shape_p));
    b->mass += mass;
    lc = vadd(lc, vscale(mass, center));
    b->I += I;
  }
  if (b->mass > 0.0f) {
    b->inv_mass = 1.0f / b->mass;
    lc = vscale(b->inv_mass, lc);
  } else {
    b->mass = 1.0f;
    b->inv_mass = 1.0f;
  }
  if (b->I > 0.0f && (b->flags & BF_FIXEDROT) == 0) {
    b->I -= b->mass * vdot(lc, lc);
    b->inv_I = 1.0f / b->I;
  } else {
    b->I = 0.0f;
    b->inv_I = 0.0f;
  }
  v2 old_center = b->c;
  b->local_center = lc;
  b->c0 = b->c = xf_mul(b->xf, b->local_center);
  b->v = vadd(b->v, vcross_sv(b->w, vsub(b->c, old_center)));
}

int b2l_create_body(b2l_world* w, const b2l_body_def* d) {
  if (w->nb == w->bcap) {
    w->bcap = w->bcap ? 2 * w->bcap : 16;
    w->bodies = (body*)xrealloc(w->bodies, sizeof(body) * w->bcap);
    w->fat = (aabb*)xrealloc(w->fat, sizeof(aabb) * w->bcap);
    w->isl_bodies = (int*)xrealloc(w->isl_bodies, sizeof(int) * w->bcap);
    w->stack = (int*)xrealloc(w->stack, sizeof(int) * w->bcap);
  }
  int id = w->nb++;
  body* b = &w->bodies[id];
  memset(b, 0, sizeof(*b));
  /* b2Body::b2Body */
  b->flags = BF_AWAKE | BF_ACTIVE;
  if (d->fixed_rotation) b->flags |= BF_FIXEDROT;
  if (d->allow_sleep) b->flags |= BF_AUTOSLEEP;
  b->xf.p = V(d->x, d->y);
  b->xf.q = rot_set(d->angle);
  b->local_center = V(0.0f, 0.0f);
  b->c0 = b->xf.p;
  b->c = b->xf.p;
  b->a0 = d->angle;
  b->a = d->angle;
  b->v = V(0.0f, 0.0f);
  b->w = 0.0f;
  b->lin_damp = d->linear_damping;
  b->ang_damp = 0.0f;
  b->gravity_scale = 1.0f;
  b->force = V(0.0f, 0.0f);
  b->torque = 0.0f;
  b->sleep_time = 0.0f;
  b->mass = 1.0f; /* dynamic body */
  b->inv_mass = 1.0f;
  b->I = 0.0f; b->inv_I = 0.0f;
  b->contact_list = -1;
  b->island_index = 0;
  /* b2World::CreateBody: prepend to the body list */
  b->prev = -1;
  b->next = w->body_list;
  if (w->body_list >= 0) w->bodies[w->body_list].prev = id;
  w->body_list = id;
  /* b2Body::CreateFixture (circle at origin) -> CreateProxies, ResetMassData */
  b->shape_p = V(0.0f, 0.0f);
  b->radius = d->radius;
  b->density = d->density;
  b->friction = d->friction;
  b->restitution = d->restitution;
  b->proxy_aabb = circle_aabb(b, b->xf);
  /* b2DynamicTree::CreateProxy: fat = aabb +- extension. Tree leaf ids are
   * allocated in creation order when no proxy was ever destroyed, so using the
   * body id as proxy id keeps every (proxyIdA, proxyIdB) comparison identical. */
  b->proxy_id = id;
  {
    v2 r = V(B2_AABB_EXTENSION, B2_AABB_EXTENSION);
    w->fat[id].lo = vsub(b->proxy_aabb.lo, r);
    w->fat[id].hi = vadd(b->proxy_aabb.hi, r);
  }
  buffer_move(w, id);
  if (b->density > 0.0f) reset_mass_data(b);
  w->new_fixture = 1;
  return id;
}

void b2l_body_get(const b2l_world* w, int id, float* o) {
  const body* b = &w->bodies[id];
  o[0] = b->xf.p.x; o[1] = b->xf.p.y; o[2] = b->a; o[3] = b->v.x; o[4] = b->v.y;
  o[5] = b->sleep_time; o[6] = (b->flags & BF_AWAKE) ? 1.0f : 0.0f;
}

void b2l_body_get_fat(const b2l_world* w, int id, float* o) {
  aabb f = w->fat[w->bodies[id].proxy_id];
  o[0] = f.lo.x; o[1] = f.lo.y; o[2] = f.hi.x; o[3] = f.hi.y;
}

/* b2DynamicTree::MoveProxy (+ b2BroadPhase::MoveProxy's BufferMove) */
static void move_proxy(b2l_world* w, int proxy, aabb bb, v2 displacement) {
  if (aabb_contains(w->fat[proxy], bb)) return;
  aabb b = bb;
  v2 r = V(B2_AABB_EXTENSION, B2_AABB_EXTENSION);
  b.lo = vsub(b.lo, r);
  b.hi = vadd(b.hi, r);
  v2 d = vscale(B2_AABB_MULTIPLIER, displacement);
  if (d.x < 0.0f) b.lo.x += d.x; else b.hi.x += d.x;
  if (d.y < 0.0f) b.lo.y += d.y; else b.hi.y += d.y;
  w->fat[proxy] = b;
  buffer_move(w, proxy);
}

/* b2Fixture::Synchronize */
static void fixture_synchronize(b2l_world* w, body* b, xform xf1, xform xf2) {
  aabb a1 = circle_aabb(b, xf1), a2 = circle_aabb(b, xf2);
  b->proxy_aabb.lo = vmin(a1.lo, a2.lo);
  b->proxy_aabb.hi = vmax(a1.hi, a2.hi);
  v2 disp = vsub(xf2.p, xf1.p);
  move_proxy(w, b->proxy_id, b->proxy_aabb, disp);
}

/* b2Body::SetTransform */
void b2l_body_set_transform(b2l_world* w, int id, float x, float y, float angle) {
  body* b = &w->bodies[id];
  b->xf.q = rot_set(angle);
  b->xf.p = V(x, y);
  b->c = xf_mul(b->xf, b->local_center);
  b->a = angle;
  b->c0 = b->c;
  b->a0 = angle;
  fixture_synchronize(w, b, b->xf, b->xf);
}

/* b2Body::SetAwake */
static void set_awake(body* b, int flag) {
  if (flag) {
    if ((b->flags & BF_AWAKE) == 0) {
      b->flags |= BF_AWAKE;
      b->sleep_time = 0.0f;
    }
  } else {
    b->flags &= ~BF_AWAKE;
    b->sleep_time = 0.0f;
    b->v = V(0.0f, 0.0f);
    b->w = 0.0f;
    b->force = V(0.0f, 0.0f);
    b->torque = 0.0f;
  }
}

/* b2Body::ApplyForce (dynamic body) */
void b2l_body_apply_force(b2l_world* w, int id, float fx, float fy, float px, float py, int wake) {
  body* b = &w->bodies[id];
  if (wake && (b->flags & BF_AWAKE) == 0) set_awake(b, 1);
  if (b->flags & BF_AWAKE) {
    v2 f = V(fx, fy);
    b->force = vadd(b->force, f);
    b->torque += vcross(vsub(V(px, py), b->c), f);
  }
}

void b2l_world_clear_forces(b2l_world* w) {
  for (int i = w->body_list; i >= 0; i = w->bodies[i].next) {
    w->bodies[i].force = V(0.0f, 0.0f);
    w->bodies[i].torque = 0.0f;
  }
}

/* ---- contact manager ---------------------------------------------------- */
static int contact_alloc(b2l_world* w) {
  if (w->free_head < 0) {
    int old = w->ccap;
    w->ccap = w->ccap ? 2 * w->ccap : 64;
    w->contacts = (contact*)xrealloc(w->contacts, sizeof(contact) * w->ccap);
    w->isl_contacts = (int*)xrealloc(w->isl_contacts, sizeof(int) * w->ccap);
    for (int i = w->ccap - 1; i >= old; --i) {
      w->contacts[i].alive = 0;
      w->contacts[i].next_free = w->free_head;
      w->free_head = i;
    }
  }
  int id = w->free_head;
  w->free_head = w->contacts[id].next_free;
  memset(&w->contacts[id], 0, sizeof(contact));
  w->contacts[id].alive = 1;
  return id;
}

static inline int edge_contact(int e) { return e >> 1; }
static inline int edge_side(int e) { return e & 1; }
static inline int edge_other(const b2l_world* w, int e) {
  const contact* c = &w->contacts[edge_contact(e)];
  return edge_side(e) == 0 ? c->fb : c->fa;
}
static inline int* edge_prev(b2l_world* w, int e) { return &w->contacts[edge_contact(e)].eprev[edge_side(e)]; }
static inline int* edge_next(b2l_world* w, int e) { return &w->contacts[edge_contact(e)].enext[edge_side(e)]; }

static void edge_prepend(b2l_world* w, int bid, int e) {
  body* b = &w->bodies[bid];
  *edge_prev(w, e) = -1;
  *edge_next(w, e) = b->contact_list;
  if (b->contact_list >= 0) *edge_prev(w, b->contact_list) = e;
  b->contact_list = e;
}

static void edge_remove(b2l_world* w, int bid, int e) {
  body* b = &w->bodies[bid];
  int p = *edge_prev(w, e), n = *edge_next(w, e);
  if (p >= 0) *edge_next(w, p) = n;
  if (n >= 0) *edge_prev(w, n) = p;
  if (b->contact_list == e) b->contact_list = n;
}

/* b2Contact::Create (circle-circle is the primary registration: no swap) +
 * the insertion half of b2ContactManager::AddPair. */
static int contact_create(b2l_world* w, int ba, int bb) {
  int id = contact_alloc(w);
  contact* c = &w->contacts[id];
  c->flags = CF_ENABLED;
  c->fa = ba;
  c->fb = bb;
  c->point_count = 0;
  /* b2MixFriction / b2MixRestitution */
  c->friction = sqrtf(w->bodies[ba].friction * w->bodies[bb].friction);
  c->restitution = fmaxb(w->bodies[ba].restitution, w->bodies[bb].restitution);
  c->tangent_speed = 0.0f;
  /* prepend to the world list */
  c->prev = -1;
  c->next = w->contact_list;
  if (w->contact_list >= 0) w->contacts[w->contact_list].prev = id;
  w->contact_list = id;
  /* connect to the island graph */
  edge_prepend(w, ba, 2 * id + 0);
  edge_prepend(w, bb, 2 * id + 1);
  ++w->contact_count;
  return id;
}

/* b2ContactManager::AddPair */
static void add_pair(b2l_world* w, int proxy_a, int proxy_b) {
  int ba = proxy_a, bb = proxy_b; /* proxy id == body id */
  if (ba == bb) return;
  /* Does a contact already exist? (walk bodyB's edge list) */
  for (int e = w->bodies[bb].contact_list; e >= 0; e = *edge_next(w, e)) {
    if (edge_other(w, e) == ba) {
      const contact* c = &w->contacts[edge_contact(e)];
      if (c->fa == ba && c->fb == bb) return;
      if (c->fa == bb && c->fb == ba) return;
    }
  }
  /* ShouldCollide: both dynamic, no joints, no filter -> true */
  contact_create(w, ba, bb);
  /* Wake up the bodies (non-sensors) */
  set_awake(&w->bodies[ba], 1);
  set_awake(&w->bodies[bb], 1);
}

static int pair_less(const void* p1, const void* p2) {
  const int* a = (const int*)p1;
  const int* b = (const int*)p2;
  if (a[0] != b[0]) return a[0] < b[0] ? -1 : 1;
  if (a[1] != b[1]) return a[1] < b[1] ? -1 : 1;
  return 0;
}

/* b2BroadPhase::UpdatePairs via b2ContactManager::FindNewContacts. The dynamic
 * tree's Query returns exactly the set of leaves whose fat AABB overlaps the
 * query AABB (internal nodes hold exact unions), so a brute-force scan over all
 * proxies yields the same pair set; the pair buffer is sorted before use. */
static void find_new_contacts(b2l_world* w) {
  w->pair_count = 0;
  for (int i = 0; i < w->move_count; ++i) {
    int q = w->move_buf[i];
    if (q < 0) continue;
    aabb qa = w->fat[q];
    for (int p = 0; p < w->nb; ++p) {
      if (p == q) continue;
      if ((w->bodies[p].flags & BF_ACTIVE) == 0) continue; /* proxy destroyed */
      if (!aabb_overlap(w->fat[p], qa)) continue;
      if (w->pair_count == w->pair_cap) {
        w->pair_cap = w->pair_cap ? 2 * w->pair_cap : 64;
        w->pair_buf = (int*)xrealloc(w->pair_buf, sizeof(int) * 2 * w->pair_cap);
      }
      w->pair_buf[2 * w->pair_count + 0] = p < q ? p : q;
      w->pair_buf[2 * w->pair_count + 1] = p < q ? q : p;
      ++w->pair_count;
    }
  }
  w->move_count = 0;
  /* qsort's base must be non-NULL even for 0 elements (the pair buffer is allocated lazily);
   * found by the sanitizer leg (tools/asan_oracle.sh) */
  if (w->pair_count > 1) qsort(w->pair_buf, (size_t)w->pair_count, 2 * sizeof(int), pair_less);
  int i = 0;
  while (i < w->pair_count) {
    int a = w->pair_buf[2 * i], b = w->pair_buf[2 * i + 1];
    add_pair(w, a, b);
    ++i;
    while (i < w->pair_count && w->pair_buf[2 * i] == a && w->pair_buf[2 * i + 1] == b) ++i;
  }
}

/* b2ContactManager::Destroy (+ b2Contact::Destroy's wake) */
static void contact_destroy(b2l_world* w, int id) {
  contact* c = &w->contacts[id];
  if (c->prev >= 0) w->contacts[c->prev].next = c->next;
  if (c->next >= 0) w->contacts[c->next].prev = c->prev;
  if (w->contact_list == id) w->contact_list = c->next;
  edge_remove(w, c->fa, 2 * id + 0);
  edge_remove(w, c->fb, 2 * id + 1);
  if (c->point_count > 0) {
    set_awake(&w->bodies[c->fa], 1);
    set_awake(&w->bodies[c->fb], 1);
  }
  c->alive = 0;
  c->next_free = w->free_head;
  w->free_head = id;
  --w->contact_count;
}

/* b2CollideCircles + b2Contact::Update (non-sensor branch) */
static void contact_update(b2l_world* w, contact* c) {
  int old_pc = c->point_count;
  float old_n = c->normal_impulse, old_t = c->tangent_impulse;
  c->flags |= CF_ENABLED;
  int was_touching = (c->flags & CF_TOUCHING) != 0;
  body* A = &w->bodies[c->fa];
  body* B = &w->bodies[c->fb];
  /* b2CollideCircles */
  int pc = 0;
  {
    v2 pA = xf_mul(A->xf, A->shape_p);
    v2 pB = xf_mul(B->xf, B->shape_p);
    v2 d = vsub(pB, pA);
    float dist_sqr = vdot(d, d);
    float radius = A->radius + B->radius;
    if (!(dist_sqr > radius * radius)) pc = 1;
  }
  c->point_count = pc;
  int touching = pc > 0;
  if (pc > 0) {
    /* match ids (key 0 == key 0) and carry impulses */
    c->normal_impulse = 0.0f;
    c->tangent_impulse = 0.0f;
    if (old_pc > 0) {
      c->normal_impulse = old_n;
      c->tangent_impulse = old_t;
    }
  }
  if (touching != was_touching) {
    set_awake(A, 1);
    set_awake(B, 1);
  }
  if (touching) c->flags |= CF_TOUCHING; else c->flags &= ~CF_TOUCHING;
  /* BeginContact / PreSolve listeners: the reference's callbacks have no effect
   * (cm_framework.py:373-408 -> mvmnt.py:250-251). */
}

/* b2ContactManager::Collide */
static void collide(b2l_world* w) {
  int ci = w->contact_list;
  while (ci >= 0) {
    contact* c = &w->contacts[ci];
    body* A = &w->bodies[c->fa];
    body* B = &w->bodies[c->fb];
    int activeA = (A->flags & BF_AWAKE) != 0;
    int activeB = (B->flags & BF_AWAKE) != 0;
    if (!activeA && !activeB) { ci = c->next; continue; }
    int overlap = aabb_overlap(w->fat[A->proxy_id], w->fat[B->proxy_id]);
    if (!overlap) {
      int nuke = ci;
      ci = c->next;
      contact_destroy(w, nuke);
      continue;
    }
    contact_update(w, c);
    ci = c->next;
  }
}

/* ---- island solver (b2Island::Solve + b2ContactSolver) ----------------- */
typedef struct { v2 c; float a; } pos_t;
typedef struct { v2 v; float w; } vel_t;

typedef struct {
  v2 rA, rB;
  float normal_impulse, tangent_impulse, normal_mass, tangent_mass, velocity_bias;
} vcpoint;

typedef struct {
  vcpoint p;
  v2 normal;
  float friction, restitution, tangent_speed;
  int ia, ib;
  float mA, mB, iA, iB;
  int contact;
} vconstraint;

typedef struct {
  int ia, ib;
  float mA, mB, iA, iB;
  v2 lcA, lcB;
  v2 local_point;   /* manifold localPoint = circleA m_p */
  v2 local_point0;  /* points[0].localPoint = circleB m_p */
  float rA, rB;     /* radii */
} pconstraint;

typedef struct {
  int nb, nc;
  int* bodies;    /* body ids in island order */
  int* contacts;  /* contact ids in island order */
  pos_t* pos;
  vel_t* vel;
  vconstraint* vc;
  pconstraint* pcs;
} island;

static void island_solve(b2l_world* w, island* isl, float h, float inv_dt, float dt_ratio,
                         int vel_iters, int pos_iters) {
  (void)inv_dt;
  /* integrate velocities, damping, init state */
  for (int i = 0; i < isl->nb; ++i) {
    body* b = &w->bodies[isl->bodies[i]];
    v2 c = b->c; float a = b->a;
    v2 v = b->v; float wv = b->w;
    b->c0 = b->c;
    b->a0 = b->a;
    /* dynamic body */
    v = vadd(v, vscale(h, vadd(vscale(b->gravity_scale, w->gravity), vscale(b->inv_mass, b->force))));
    wv += h * b->inv_I * b->torque;
    v = vscale(1.0f / (1.0f + h * b->lin_damp), v);
    wv *= 1.0f / (1.0f + h * b->ang_damp);
    isl->pos[i].c = c; isl->pos[i].a = a;
    isl->vel[i].v = v; isl->vel[i].w = wv;
  }

  /* b2ContactSolver::b2ContactSolver */
  for (int i = 0; i < isl->nc; ++i) {
    contact* ct = &w->contacts[isl->contacts[i]];
    body* A = &w->bodies[ct->fa];
    body* B = &w->bodies[ct->fb];
    vconstraint* vc = &isl->vc[i];
    pconstraint* pc = &isl->pcs[i];
    vc->friction = ct->friction;
    vc->restitution = ct->restitution;
    vc->tangent_speed = ct->tangent_speed;
    vc->ia = A->island_index; vc->ib = B->island_index;
    vc->mA = A->inv_mass; vc->mB = B->inv_mass; vc->iA = A->inv_I; vc->iB = B->inv_I;
    vc->contact = isl->contacts[i];
    pc->ia = A->island_index; pc->ib = B->island_index;
    pc->mA = A->inv_mass; pc->mB = B->inv_mass;
    pc->lcA = A->local_center; pc->lcB = B->local_center;
    pc->iA = A->inv_I; pc->iB = B->inv_I;
    pc->local_point = A->shape_p;
    pc->local_point0 = B->shape_p;
    pc->rA = A->radius; pc->rB = B->radius;
    /* one manifold point */
    if (w->warm_starting) {
      vc->p.normal_impulse = dt_ratio * ct->normal_impulse;
      vc->p.tangent_impulse = dt_ratio * ct->tangent_impulse;
    } else {
      vc->p.normal_impulse = 0.0f;
      vc->p.tangent_impulse = 0.0f;
    }
    vc->p.rA = V(0.0f, 0.0f); vc->p.rB = V(0.0f, 0.0f);
    vc->p.normal_mass = 0.0f; vc->p.tangent_mass = 0.0f; vc->p.velocity_bias = 0.0f;
  }

  /* InitializeVelocityConstraints (b2WorldManifold::Initialize, e_circles) */
  for (int i = 0; i < isl->nc; ++i) {
    vconstraint* vc = &isl->vc[i];
    pconstraint* pc = &isl->pcs[i];
    float mA = vc->mA, mB = vc->mB, iA = vc->iA, iB = vc->iB;
    v2 cA = isl->pos[vc->ia].c; float aA = isl->pos[vc->ia].a;
    v2 vA = isl->vel[vc->ia].v; float wA = isl->vel[vc->ia].w;
    v2 cB = isl->pos[vc->ib].c; float aB = isl->pos[vc->ib].a;
    v2 vB = isl->vel[vc->ib].v; float wB = isl->vel[vc->ib].w;
    xform xfA, xfB;
    xfA.q = rot_set(aA); xfB.q = rot_set(aB);
    xfA.p = vsub(cA, rot_mul(xfA.q, pc->lcA));
    xfB.p = vsub(cB, rot_mul(xfB.q, pc->lcB));
    v2 normal = V(1.0f, 0.0f);
    v2 pointA = xf_mul(xfA, pc->local_point);
    v2 pointB = xf_mul(xfB, pc->local_point0);
    if (vdist2(pointA, pointB) > B2_EPS * B2_EPS) {
      normal = vsub(pointB, pointA);
      vnormalize(&normal);
    }
    v2 wcA = vadd(pointA, vscale(pc->rA, normal));
    v2 wcB = vsub(pointB, vscale(pc->rB, normal));
    v2 wpoint = vscale(0.5f, vadd(wcA, wcB));
    vc->normal = normal;
    vcpoint* vcp = &vc->p;
    vcp->rA = vsub(wpoint, cA);
    vcp->rB = vsub(wpoint, cB);
    float rnA = vcross(vcp->rA, vc->normal);
    float rnB = vcross(vcp->rB, vc->normal);
    float kNormal = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
    vcp->normal_mass = kNormal > 0.0f ? 1.0f / kNormal : 0.0f;
    v2 tangent = vcross_vs(vc->normal, 1.0f);
    float rtA = vcross(vcp->rA, tangent);
    float rtB = vcross(vcp->rB, tangent);
    float kTangent = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
    vcp->tangent_mass = kTangent > 0.0f ? 1.0f / kTangent : 0.0f;
    vcp->velocity_bias = 0.0f;
    float vRel = vdot(vc->normal, vsub(vsub(vadd(vB, vcross_sv(wB, vcp->rB)), vA), vcross_sv(wA, vcp->rA)));
    if (vRel < -B2_VELOCITY_THRESHOLD) vcp->velocity_bias = -vc->restitution * vRel;
  }

  /* WarmStart */
  if (w->warm_starting) {
    for (int i = 0; i < isl->nc; ++i) {
      vconstraint* vc = &isl->vc[i];
      float mA = vc->mA, iA = vc->iA, mB = vc->mB, iB = vc->iB;
      v2 vA = isl->vel[vc->ia].v; float wA = isl->vel[vc->ia].w;
      v2 vB = isl->vel[vc->ib].v; float wB = isl->vel[vc->ib].w;
      v2 normal = vc->normal;
      v2 tangent = vcross_vs(normal, 1.0f);
      vcpoint* vcp = &vc->p;
      v2 P = vadd(vscale(vcp->normal_impulse, normal), vscale(vcp->tangent_impulse, tangent));
      wA -= iA * vcross(vcp->rA, P);
      vA = vsub(vA, vscale(mA, P));
      wB += iB * vcross(vcp->rB, P);
      vB = vadd(vB, vscale(mB, P));
      isl->vel[vc->ia].v = vA; isl->vel[vc->ia].w = wA;
      isl->vel[vc->ib].v = vB; isl->vel[vc->ib].w = wB;
    }
  }

  /* SolveVelocityConstraints x vel_iters */
  for (int it = 0; it < vel_iters; ++it) {
    for (int i = 0; i < isl->nc; ++i) {
      vconstraint* vc = &isl->vc[i];
      float mA = vc->mA, iA = vc->iA, mB = vc->mB, iB = vc->iB;
      v2 vA = isl->vel[vc->ia].v; float wA = isl->vel[vc->ia].w;
      v2 vB = isl->vel[vc->ib].v; float wB = isl->vel[vc->ib].w;
      v2 normal = vc->normal;
      v2 tangent = vcross_vs(normal, 1.0f);
      float friction = vc->friction;
      vcpoint* vcp = &vc->p;
      {
        v2 dv = vsub(vsub(vadd(vB, vcross_sv(wB, vcp->rB)), vA), vcross_sv(wA, vcp->rA));
        float vt = vdot(dv, tangent) - vc->tangent_speed;
        float lambda = vcp->tangent_mass * (-vt);
        float maxFriction = friction * vcp->normal_impulse;
        float newImpulse = fclampb(vcp->tangent_impulse + lambda, -maxFriction, maxFriction);
        lambda = newImpulse - vcp->tangent_impulse;
        vcp->tangent_impulse = newImpulse;
        v2 P = vscale(lambda, tangent);
        vA = vsub(vA, vscale(mA, P));
        wA -= iA * vcross(vcp->rA, P);
        vB = vadd(vB, vscale(mB, P));
        wB += iB * vcross(vcp->rB, P);
      }
      {
        v2 dv = vsub(vsub(vadd(vB, vcross_sv(wB, vcp->rB)), vA), vcross_sv(wA, vcp->rA));
        float vn = vdot(dv, normal);
        float lambda = -vcp->normal_mass * (vn - vcp->velocity_bias);
        float newImpulse = fmaxb(vcp->normal_impulse + lambda, 0.0f);
        lambda = newImpulse - vcp->normal_impulse;
        vcp->normal_impulse = newImpulse;
        v2 P = vscale(lambda, normal);
        vA = vsub(vA, vscale(mA, P));
        wA -= iA * vcross(vcp->rA, P);
        vB = vadd(vB, vscale(mB, P));
        wB += iB * vcross(vcp->rB, P);
      }
      isl->vel[vc->ia].v = vA; isl->vel[vc->ia].w = wA;
      isl->vel[vc->ib].v = vB; isl->vel[vc->ib].w = wB;
    }
  }

  /* StoreImpulses */
  for (int i = 0; i < isl->nc; ++i) {
    contact* ct = &w->contacts[isl->vc[i].contact];
    ct->normal_impulse = isl->vc[i].p.normal_impulse;
    ct->tangent_impulse = isl->vc[i].p.tangent_impulse;
  }

  /* integrate positions */
  for (int i = 0; i < isl->nb; ++i) {
    v2 c = isl->pos[i].c; float a = isl->pos[i].a;
    v2 v = isl->vel[i].v; float wv = isl->vel[i].w;
    v2 translation = vscale(h, v);
    if (vdot(translation, translation) > B2_MAX_TRANSLATION_SQ) {
      float ratio = B2_MAX_TRANSLATION / vlen(translation);
      v = vscale(ratio, v);
    }
    float rotation = h * wv;
    if (rotation * rotation > B2_MAX_ROTATION_SQ) {
      float ratio = B2_MAX_ROTATION / fabsf(rotation);
      wv *= ratio;
    }
    c = vadd(c, vscale(h, v));
    a += h * wv;
    isl->pos[i].c = c; isl->pos[i].a = a;
    isl->vel[i].v = v; isl->vel[i].w = wv;
  }

  /* SolvePositionConstraints (b2PositionSolverManifold, e_circles) */
  int position_solved = 0;
  for (int it = 0; it < pos_iters; ++it) {
    float minSeparation = 0.0f;
    for (int i = 0; i < isl->nc; ++i) {
      pconstraint* pc = &isl->pcs[i];
      float mA = pc->mA, iA = pc->iA, mB = pc->mB, iB = pc->iB;
      v2 cA = isl->pos[pc->ia].c; float aA = isl->pos[pc->ia].a;
      v2 cB = isl->pos[pc->ib].c; float aB = isl->pos[pc->ib].a;
      xform xfA, xfB;
      xfA.q = rot_set(aA); xfB.q = rot_set(aB);
      xfA.p = vsub(cA, rot_mul(xfA.q, pc->lcA));
      xfB.p = vsub(cB, rot_mul(xfB.q, pc->lcB));
      v2 pointA = xf_mul(xfA, pc->local_point);
      v2 pointB = xf_mul(xfB, pc->local_point0);
      v2 normal = vsub(pointB, pointA);
      vnormalize(&normal);
      v2 point = vscale(0.5f, vadd(pointA, pointB));
      float separation = vdot(vsub(pointB, pointA), normal) - pc->rA - pc->rB;
      v2 rA = vsub(point, cA), rB = vsub(point, cB);
      minSeparation = fminb(minSeparation, separation);
      float C = fclampb(B2_BAUMGARTE * (separation + B2_LINEAR_SLOP), -B2_MAX_LINEAR_CORRECTION, 0.0f);
      float rnA = vcross(rA, normal), rnB = vcross(rB, normal);
      float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      float impulse = K > 0.0f ? -C / K : 0.0f;
      v2 P = vscale(impulse, normal);
      cA = vsub(cA, vscale(mA, P));
      aA -= iA * vcross(rA, P);
      cB = vadd(cB, vscale(mB, P));
      aB += iB * vcross(rB, P);
      isl->pos[pc->ia].c = cA; isl->pos[pc->ia].a = aA;
      isl->pos[pc->ib].c = cB; isl->pos[pc->ib].a = aB;
    }
    if (minSeparation >= -3.0f * B2_LINEAR_SLOP) { position_solved = 1; break; }
  }

  /* copy back + SynchronizeTransform */
  for (int i = 0; i < isl->nb; ++i) {
    body* b = &w->bodies[isl->bodies[i]];
    b->c = isl->pos[i].c; b->a = isl->pos[i].a;
    b->v = isl->vel[i].v; b->w = isl->vel[i].w;
    b->xf.q = rot_set(b->a);
    b->xf.p = vsub(b->c, rot_mul(b->xf.q, b->local_center));
  }

  /* sleep */
  if (w->allow_sleep) {
    float minSleepTime = FLT_MAX;
    const float linTolSqr = B2_LINEAR_SLEEP_TOL * B2_LINEAR_SLEEP_TOL;
    const float angTolSqr = B2_ANGULAR_SLEEP_TOL * B2_ANGULAR_SLEEP_TOL;
    for (int i = 0; i < isl->nb; ++i) {
      body* b = &w->bodies[isl->bodies[i]];
      if ((b->flags & BF_AUTOSLEEP) == 0 || b->w * b->w > angTolSqr || vdot(b->v, b->v) > linTolSqr) {
        b->sleep_time = 0.0f;
        minSleepTime = 0.0f;
      } else {
        b->sleep_time += h;
        minSleepTime = fminb(minSleepTime, b->sleep_time);
      }
    }
    if (minSleepTime >= B2_TIME_TO_SLEEP && position_solved) {
      for (int i = 0; i < isl->nb; ++i) set_awake(&w->bodies[isl->bodies[i]], 0);
    }
  }
}

/* b2Body::SynchronizeFixtures */
static void synchronize_fixtures(b2l_world* w, body* b) {
  xform xf1;
  xf1.q = rot_set(b->a0);
  xf1.p = vsub(b->c0, rot_mul(xf1.q, b->local_center));
  fixture_synchronize(w, b, xf1, b->xf);
}

/* b2World::Solve */
static void world_solve(b2l_world* w, float h, float inv_dt, float dt_ratio, int vel_iters,
                        int pos_iters) {
  for (int i = w->body_list; i >= 0; i = w->bodies[i].next) w->bodies[i].flags &= ~BF_ISLAND;
  for (int c = w->contact_list; c >= 0; c = w->contacts[c].next) w->contacts[c].flags &= ~CF_ISLAND;

  island isl;
  isl.bodies = w->isl_bodies;
  isl.contacts = w->isl_contacts;
  isl.pos = (pos_t*)malloc(sizeof(pos_t) * (size_t)(w->nb ? w->nb : 1));
  isl.vel = (vel_t*)malloc(sizeof(vel_t) * (size_t)(w->nb ? w->nb : 1));
  int ncap = w->contact_count ? w->contact_count : 1;
  isl.vc = (vconstraint*)malloc(sizeof(vconstraint) * (size_t)ncap);
  isl.pcs = (pconstraint*)malloc(sizeof(pconstraint) * (size_t)ncap);
  int* stack = w->stack;

  for (int seed = w->body_list; seed >= 0; seed = w->bodies[seed].next) {
    body* sb = &w->bodies[seed];
    if (sb->flags & BF_ISLAND) continue;
    if ((sb->flags & BF_AWAKE) == 0 || (sb->flags & BF_ACTIVE) == 0) continue;
    isl.nb = 0;
    isl.nc = 0;
    int sp = 0;
    stack[sp++] = seed;
    sb->flags |= BF_ISLAND;
    while (sp > 0) {
      int bi = stack[--sp];
      body* b = &w->bodies[bi];
      b->island_index = isl.nb;
      isl.bodies[isl.nb++] = bi;
      set_awake(b, 1);
      for (int e = b->contact_list; e >= 0; e = *edge_next(w, e)) {
        int ci = edge_contact(e);
        contact* c = &w->contacts[ci];
        if (c->flags & CF_ISLAND) continue;
        if ((c->flags & CF_ENABLED) == 0 || (c->flags & CF_TOUCHING) == 0) continue;
        isl.contacts[isl.nc++] = ci;
        c->flags |= CF_ISLAND;
        int other = edge_other(w, e);
        body* ob = &w->bodies[other];
        if (ob->flags & BF_ISLAND) continue;
        stack[sp++] = other;
        ob->flags |= BF_ISLAND;
      }
    }
    island_solve(w, &isl, h, inv_dt, dt_ratio, vel_iters, pos_iters);
  }
  free(isl.pos); free(isl.vel); free(isl.vc); free(isl.pcs);

  for (int i = w->body_list; i >= 0; i = w->bodies[i].next) {
    body* b = &w->bodies[i];
    if ((b->flags & BF_ISLAND) == 0) continue;
    synchronize_fixtures(w, b);
  }
  find_new_contacts(w);
}

/* b2World::Step. SolveTOI is provably a no-op for this workload: it only
 * considers pairs where one body is static/kinematic or a bullet, and every
 * body here is a non-bullet dynamic body. */
void b2l_world_step(b2l_world* w, float dt, int vel_iters, int pos_iters) {
  if (w->new_fixture) {
    find_new_contacts(w);
    w->new_fixture = 0;
  }
  float inv_dt = dt > 0.0f ? 1.0f / dt : 0.0f;
  float dt_ratio = w->inv_dt0 * dt;
  collide(w);
  if (w->step_complete && dt > 0.0f) world_solve(w, dt, inv_dt, dt_ratio, vel_iters, pos_iters);
  if (dt > 0.0f) w->inv_dt0 = inv_dt;
  /* m_flags & e_clearForces (autoClearForces default true) */
  b2l_world_clear_forces(w);
}

int b2l_world_contacts(const b2l_world* w, int* out, int cap) {
  int n = 0;
  for (int c = w->contact_list; c >= 0; c = w->contacts[c].next) {
    if (n < cap) {
      out[3 * n + 0] = w->contacts[c].fa;
      out[3 * n + 1] = w->contacts[c].fb;
      out[3 * n + 2] = (w->contacts[c].flags & CF_TOUCHING) ? 1 : 0;
    }
    ++n;
  }
  return n;
}

int b2l_world_contact_impulses(const b2l_world* w, float* out, int cap) {
  int n = 0;
  for (int c = w->contact_list; c >= 0; c = w->contacts[c].next) {
    if (n < cap) {
      out[3 * n + 0] = w->contacts[c].normal_impulse;
      out[3 * n + 1] = w->contacts[c].tangent_impulse;
      out[3 * n + 2] = (float)w->contacts[c].point_count;
    }
    ++n;
  }
  return n;
}

void b2l_world_load_contacts(b2l_world* w, int n, const int* ab, const float* imp,
                             const int* point_count) {
  /* drop everything */
  while (w->contact_list >= 0) {
    int c = w->contact_list;
    w->contacts[c].point_count = 0; /* no wake side effects needed */
    contact_destroy(w, c);
  }
  /* re-create tail first so that prepending reproduces the given order */
  for (int k = n - 1; k >= 0; --k) {
    int id = contact_create(w, ab[2 * k], ab[2 * k + 1]);
    contact* c = &w->contacts[id];
    c->point_count = point_count ? point_count[k] : 0;
    c->normal_impulse = imp ? imp[2 * k] : 0.0f;
    c->tangent_impulse = imp ? imp[2 * k + 1] : 0.0f;
    if (c->point_count > 0) c->flags |= CF_TOUCHING;
  }
  w->move_count = 0;
}

void b2l_body_set_state(b2l_world* w, int id, float x, float y, float angle, float vx, float vy,
                        float sleep_time, const float* fat4) {
  body* b = &w->bodies[id];
  b->xf.p = V(x, y);
  b->xf.q = rot_set(angle);
  b->c = b->c0 = b->xf.p;
  b->a = b->a0 = angle;
  b->v = V(vx, vy);
  b->sleep_time = sleep_time;
  b->flags |= BF_AWAKE;
  if (fat4) {
    w->fat[b->proxy_id].lo = V(fat4[0], fat4[1]);
    w->fat[b->proxy_id].hi = V(fat4[2], fat4[3]);
  }
}

/* Run the FindNewContacts that b2World::Step performs first when new fixtures
 * exist (e_newFixture). Doing it before the step is equivalent: the step would
 * run it on the same fat AABBs before Collide. */
void b2l_world_flush_new_contacts(b2l_world* w) {
  if (w->new_fixture) {
    find_new_contacts(w);
    w->new_fixture = 0;
  }
}

/* b2Body::SetActive(false): DestroyProxies (+ UnBufferMove) and destroy every
 * attached contact. Reactivation is not needed by the reference (TDM deaths,
 * gym_macm/envs/combat.py:157-165). */
void b2l_body_set_active(b2l_world* w, int id, int flag) {
  body* b = &w->bodies[id];
  if (flag || (b->flags & BF_ACTIVE) == 0) return;
  b->flags &= ~BF_ACTIVE;
  for (int i = 0; i < w->move_count; ++i)
    if (w->move_buf[i] == b->proxy_id) w->move_buf[i] = -1;
  int e = b->contact_list;
  while (e >= 0) {
    int next = *edge_next(w, e);
    contact_destroy(w, edge_contact(e));
    e = next;
  }
  b->contact_list = -1;
}

int b2l_body_active(const b2l_world* w, int id) { return (w->bodies[id].flags & BF_ACTIVE) != 0; }

/* b2World::RayCast with a closest-hit callback that returns the reported
 * fraction (cm_framework.py:56-86): b2CircleShape::RayCast per proxy with the
 * clipped maxFraction. The dynamic tree visits candidates in a tree-dependent
 * order; only exactly equal fractions could make that order matter, and here
 * candidates are visited in proxy order. Returns the body of the last reported
 * fixture (= closest hit) or -1. */
int b2l_world_raycast(const b2l_world* w, float x1, float y1, float x2, float y2, float* fraction_out) {
  float max_fraction = 1.0f;
  int best = -1;
  v2 p1 = V(x1, y1), p2 = V(x2, y2);
  for (int i = 0; i < w->nb; ++i) {
    const body* b = &w->bodies[i];
    if ((b->flags & BF_ACTIVE) == 0) continue;
    v2 position = vadd(b->xf.p, rot_mul(b->xf.q, b->shape_p));
    v2 s = vsub(p1, position);
    float bb = vdot(s, s) - b->radius * b->radius;
    v2 r = vsub(p2, p1);
    float c = vdot(s, r);
    float rr = vdot(r, r);
    float sigma = c * c - rr * bb;
    if (sigma < 0.0f || rr < B2_EPS) continue;
    float a = -(c + sqrtf(sigma));
    if (0.0f <= a && a <= max_fraction * rr) {
      a /= rr;
      max_fraction = a; /* ReportFixture returns fraction */
      best = i;
    }
  }
  if (fraction_out) *fraction_out = max_fraction;
  return best;
}

void b2l_world_set_solver_state(b2l_world* w, float inv_dt0, int new_fixture) {
  w->inv_dt0 = inv_dt0;
  w->new_fixture = new_fixture;
  if (!new_fixture) w->move_count = 0;
}
