"""Analytic known-answer tests for the oracle's Box2D 2.3 restatement (b2lite).

Box2D itself is absent from this container, so its dynamics cannot be pinned
against it ("parity unpinned"). These tests pin the restatement
to closed-form consequences of Box2D 2.3's published algorithm, computed here
independently in numpy float32 (SURVEY.md §8(c) list, Appendix A)."""
import numpy as np

from oracle import B2World

f32 = np.float32
DT = f32(1.0 / 60.0)
INV_M = f32(1.0) / (f32(1.0) * f32(3.14159265359) * f32(0.5) * f32(0.5))
DAMP = f32(1.0) / (f32(1.0) + DT * f32(5.0))


def world_with(bodies, damping=5.0):
    w = B2World()
    for (x, y) in bodies:
        w.create_body(x, y, 0.0, 0.5, 1.0, 0.3, damping, True)
    return w


def test_constants():
    assert DT == f32(0.016666668)
    assert INV_M == f32(1.2732395)
    assert DAMP == f32(0.92307687)
    # dtRatio = fl32(fl32(1/dt) * dt) == 1 exactly: warm-start impulses carry over unscaled
    assert f32(f32(1.0) / DT) * DT == f32(1.0)


def test_free_body_velocity_sequence_bit_exact():
    """v_{k+1} = fl32(fl32(v_k + h*(0 + invM*F)) * d), x_{k+1} = x_k + h*v_{k+1}."""
    w = world_with([(0.0, 0.0)])
    F = f32(20.0)
    v = f32(0.0)
    x = f32(0.0)
    for k in range(200):
        w.apply_force(0, float(F), 0.0, *w.body(0)[:2], True)
        w.step(float(DT), 8, 3)
        w.clear_forces()
        v = f32(f32(v + DT * f32(f32(0.0) + INV_M * F)) * DAMP)
        x = f32(x + DT * v)
        s = w.body(0)
        assert f32(s[3]) == v and f32(s[0]) == x, k
    # terminal speed F*invM*h*d/(1-d) ~= 5.09 m/s
    assert abs(float(v) - float(F * INV_M * DT * DAMP / (1 - DAMP))) < 1e-4


def test_sleep_after_half_second_at_rest():
    """sleepTime accumulates h while |v|^2 <= 0.01^2; the island sleeps (v := 0,
    sleepTime := 0) once it reaches 0.5 s: fl32 sum of 30 steps = 0.5000002."""
    w = world_with([(0.0, 0.0)])
    acc = f32(0.0)
    for k in range(1, 31):
        w.step(float(DT), 8, 3)
        acc = f32(acc + DT)
        s = w.body(0)
        if k < 30:
            assert f32(s[5]) == acc and s[6] == 1.0
    assert acc >= f32(0.5)
    s = w.body(0)
    assert s[5] == 0.0 and s[6] == 0.0  # asleep, clock reset


def test_moving_body_does_not_sleep():
    w = world_with([(0.0, 0.0)])
    for _ in range(40):
        w.apply_force(0, 20.0, 0.0, *w.body(0)[:2], True)
        w.step(float(DT), 8, 3)
        w.clear_forces()
    assert w.body(0)[5] == 0.0 and w.body(0)[6] == 1.0


def test_head_on_overlap_position_correction():
    """Two resting circles 0.9 apart: relative velocity 0, so the velocity solver
    applies nothing; the position solver pushes each by mA*(-C/K) along the normal,
    C = clamp(0.2*(sep + 0.005), -0.2, 0), iterating while minSep < -0.015 (<= 3 x)."""
    w = world_with([(-0.45, 0.0), (0.45, 0.0)])
    w.step(float(DT), 8, 3)
    xa, xb = f32(-0.45), f32(0.45)
    K = INV_M + INV_M
    for _ in range(3):
        d = f32(xb - xa)
        n = f32(d * (f32(1.0) / f32(np.sqrt(f32(d * d + f32(0.0) * f32(0.0))))))  # normalize((d, 0))
        sep = f32(f32(f32(d * n + f32(0.0) * f32(0.0)) - f32(0.5)) - f32(0.5))
        C = min(max(f32(f32(0.2) * f32(sep + f32(0.005))), f32(-0.2)), f32(0.0))
        imp = f32(-C / K)
        P = f32(imp * n)
        xa = f32(xa - f32(INV_M * P))
        xb = f32(xb + f32(INV_M * P))
        if sep >= f32(-0.015):
            break
    sa, sb = w.body(0), w.body(1)
    assert f32(sa[0]) == xa and f32(sb[0]) == xb
    assert sa[1] == 0.0 and sb[1] == 0.0
    assert xb - xa > 0.9


def test_fat_aabb_hysteresis():
    """A resting body keeps its creation fat AABB (tight +- 0.1); a body that leaves
    it gets combined swept AABB +- 0.1, extended by 2*displacement on the motion side."""
    from oracle import lib
    import ctypes
    L = lib()
    w = world_with([(0.0, 0.0)])
    fat = (ctypes.c_float * 4)()
    L.b2l_body_get_fat(w.h, 0, fat)
    assert [f32(v) for v in fat] == [f32(f32(0.0 - 0.5) - f32(0.1)), f32(f32(0.0 - 0.5) - f32(0.1)),
                                     f32(f32(0.0 + 0.5) + f32(0.1)), f32(f32(0.0 + 0.5) + f32(0.1))]
    x0 = f32(0.0)
    moved = False
    for _ in range(60):
        w.apply_force(0, 20.0, 0.0, *w.body(0)[:2], True)
        prev = [f32(v) for v in fat]
        w.step(float(DT), 8, 3)
        w.clear_forces()
        x1 = f32(w.body(0)[0])
        L.b2l_body_get_fat(w.h, 0, fat)
        now = [f32(v) for v in fat]
        lo, hi = min(f32(x0 - f32(0.5)), f32(x1 - f32(0.5))), max(f32(x0 + f32(0.5)), f32(x1 + f32(0.5)))
        if prev[0] <= lo and hi <= prev[2]:
            assert now == prev
        else:
            moved = True
            d = f32(f32(2.0) * f32(x1 - x0))
            assert now[0] == f32(lo - f32(0.1)) and now[2] == f32(f32(hi + f32(0.1)) + d)
        x0 = x1
    assert moved


def test_contact_list_is_fat_aabb_overlap_not_touching():
    """SURVEY.md semantic trap #1: world.contacts holds every pair whose fat AABBs
    overlap (half-extent 0.6 at rest), so two agents 1.15 apart are 'colliding' for
    the reward although the circles (radius 0.5) do not touch; 1.25 apart are not."""
    w = world_with([(0.0, 0.0), (1.15, 0.0), (10.0, 0.0), (11.25, 0.0)])
    w.step(float(DT), 8, 3)
    c = w.contacts()
    assert [(a, b) for a, b, _ in c] == [(0, 1)]
    assert c[0][2] == 0  # not touching
