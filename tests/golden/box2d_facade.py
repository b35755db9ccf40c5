"""`Box2D` facade used ONLY by make_golden.py to run the reference's env code.

pybox2d is not installed here. This module exposes the names the reference
imports (cm_framework.py:28-33, mvmnt.py:4-5, settings.py:109, combat.py:4-5) and
implements the members the Flock hot path touches with pybox2d's observable
semantics, backed by the oracle's b2lite world (oracle/b2lite.c):
  * b2Vec2 stores float32; `a - b` is a float32 subtraction; indexing returns the
    float32 value as a Python float (pybox2d/SWIG behaviour).
  * b2DistanceSquared computes (a-b).(a-b) in float32 (b2Math.h).
  * body.angle getter = m_sweep.a; setter = SetTransform(position, float32(angle)).
  * body.ApplyForce(force, point, wake) converts the force to float32.
  * world.Step(dt, vi, pi) converts dt to float32 (SWIG float argument).
  * world.contacts lists every contact of the world list (touching or not), in
    world-list order, with fixtureA/fixtureB.body.userData.
The physics behind it is therefore the oracle's restatement, NOT real Box2D: the
golden vectors made through this facade pin the reference's env layer
(RNG/init order, action->force/angle arithmetic, reward and observation logic,
done timing), not Box2D's dynamics.
"""
import sys
import types

import numpy as np

f32 = np.float32


class b2Vec2(object):
    __slots__ = ("x", "y")

    def __init__(self, x=0.0, y=None):
        if y is None:
            x, y = x
        self.x = f32(x)
        self.y = f32(y)

    def __sub__(self, o):
        o = o if isinstance(o, b2Vec2) else b2Vec2(o)
        return b2Vec2(f32(self.x - o.x), f32(self.y - o.y))

    def __add__(self, o):
        # pybox2d: b2Vec2 __add__(b2Vec2*) in C++, a tuple converted to float32 first
        o = o if isinstance(o, b2Vec2) else b2Vec2(o)
        return b2Vec2(f32(self.x + o.x), f32(self.y + o.y))

    def __getitem__(self, i):
        return float((self.x, self.y)[i])

    def __iter__(self):
        return iter((float(self.x), float(self.y)))

    def __len__(self):
        return 2

    def __repr__(self):
        return "b2Vec2(%r,%r)" % (float(self.x), float(self.y))


def b2DistanceSquared(a, b):
    a = a if isinstance(a, b2Vec2) else b2Vec2(a)
    b = b if isinstance(b, b2Vec2) else b2Vec2(b)
    cx = f32(a.x - b.x)
    cy = f32(a.y - b.y)
    return float(f32(f32(cx * cx) + f32(cy * cy)))


class b2Color(object):
    def __init__(self, *a):
        self.rgb = a


class b2CircleShape(object):
    def __init__(self, radius=0.5, pos=(0, 0)):
        self.radius = radius


class b2FixtureDef(object):
    def __init__(self, shape=None, density=0.0, friction=0.2, restitution=0.0, isSensor=False):
        self.shape = shape
        self.density = density
        self.friction = friction
        self.restitution = restitution


class _Stub(object):
    def __init__(self, *a, **k):
        pass


class b2ContactListener(_Stub):
    pass


class b2DestructionListener(_Stub):
    pass


class b2RayCastCallback(_Stub):
    pass


class b2QueryCallback(_Stub):
    pass


class b2DrawExtended(_Stub):
    pass


class b2Fixture(_Stub):
    pass


class b2Joint(_Stub):
    pass


class b2AABB(_Stub):
    pass


class b2EdgeShape(_Stub):
    pass


class b2PolygonShape(_Stub):
    pass


def b2GetPointStates(*a):
    raise NotImplementedError


def b2Random(*a):
    raise NotImplementedError


b2_addState = 1
b2_persistState = 2
b2_dynamicBody = 2
b2_epsilon = float(np.finfo(np.float32).eps)


class _Fixture(object):
    def __init__(self, body):
        self.body = body


class _Contact(object):
    __slots__ = ("fixtureA", "fixtureB", "touching")

    def __init__(self, a, b, touching):
        self.fixtureA = _Fixture(a)
        self.fixtureB = _Fixture(b)
        self.touching = bool(touching)


class b2Body(object):
    def __init__(self, world, idx, userData):
        self._w = world
        self._i = idx
        self.userData = userData

    @property
    def position(self):
        s = self._w._core.body(self._i)
        return b2Vec2(s[0], s[1])

    @property
    def angle(self):
        return float(self._w._core.body(self._i)[2])

    @angle.setter
    def angle(self, value):
        p = self.position
        self._w._core.set_transform(self._i, float(p.x), float(p.y), float(f32(value)))

    @property
    def linearVelocity(self):
        s = self._w._core.body(self._i)
        return b2Vec2(s[3], s[4])

    @property
    def active(self):
        return bool(self._w._core.active(self._i))

    @active.setter
    def active(self, flag):
        self._w._core.set_active(self._i, bool(flag))

    def ApplyForce(self, force, point, wake):
        fx, fy = force
        p = point if isinstance(point, b2Vec2) else b2Vec2(point)
        self._w._core.apply_force(self._i, float(f32(fx)), float(f32(fy)), float(p.x), float(p.y), wake)


class b2World(object):
    def __init__(self, gravity=(0, 0), doSleep=True):
        assert tuple(gravity) == (0, 0) and doSleep, "facade models the reference's world only"
        from oracle import B2World  # oracle/oracle.py
        self._core = B2World()
        self._bodies = []
        self.contactListener = None
        self.destructionListener = None
        self.warmStarting = True
        self.continuousPhysics = True
        self.subStepping = False

    def CreateDynamicBody(self, fixtures, position, angle=0.0, linearDamping=0.0, fixedRotation=False,
                          userData=None):
        shape = fixtures.shape
        idx = self._core.create_body(float(f32(position[0])), float(f32(position[1])), float(f32(angle)),
                                     float(f32(shape.radius)), float(f32(fixtures.density)),
                                     float(f32(fixtures.friction)), float(f32(linearDamping)), fixedRotation)
        b = b2Body(self, idx, userData)
        self._bodies.append(b)
        return b

    def Step(self, timeStep, velocityIterations, positionIterations):
        self._core.step(float(f32(timeStep)), int(velocityIterations), int(positionIterations),
                        self.warmStarting, self.continuousPhysics, self.subStepping)

    def ClearForces(self):
        self._core.clear_forces()

    def RayCast(self, callback, point1, point2):
        """b2World::RayCast; the oracle returns the closest hit, which is the
        fixture a fraction-returning callback ends on (cm_framework.py:56-86)."""
        p1 = point1 if isinstance(point1, b2Vec2) else b2Vec2(point1)
        p2 = point2 if isinstance(point2, b2Vec2) else b2Vec2(point2)
        hit, fraction = self._core.raycast(float(p1.x), float(p1.y), float(p2.x), float(p2.y))
        if hit >= 0:
            fr = f32(fraction)
            point = b2Vec2(f32(f32(f32(1.0) - fr) * p1.x + fr * p2.x), f32(f32(f32(1.0) - fr) * p1.y + fr * p2.y))
            callback.ReportFixture(_Fixture(self._bodies[hit]), point, b2Vec2(0.0, 0.0), float(fr))

    @property
    def contacts(self):
        return [_Contact(self._bodies[a], self._bodies[b], t) for a, b, t in self._core.contacts()]


def install():
    m = types.ModuleType("Box2D")
    g = globals()
    for name in ("b2Vec2", "b2DistanceSquared", "b2Color", "b2CircleShape", "b2FixtureDef",
                 "b2ContactListener", "b2DestructionListener", "b2RayCastCallback", "b2QueryCallback",
                 "b2DrawExtended", "b2Fixture", "b2Joint", "b2AABB", "b2EdgeShape", "b2PolygonShape",
                 "b2GetPointStates", "b2Random", "b2_addState", "b2_persistState", "b2_dynamicBody",
                 "b2_epsilon", "b2World", "b2Body"):
        setattr(m, name, g[name])
    sys.modules["Box2D"] = m
