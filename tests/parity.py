"""Helpers comparing the HIP world against the CPU oracle (tests/ only)."""
import numpy as np

from oracle import OracleFlock

STATE_KEYS = ("pos", "vel", "angle", "fat", "sleep", "targets", "step_count", "time_passed")


def assert_state_equal(gs, os_, ctx=""):
    """Bit-exact state equality (numpy ==, so -0.0 == +0.0; see flock_step_w64.hip
    'Exactness notes' for why signed zeros of velocity may differ)."""
    for k in STATE_KEYS:
        np.testing.assert_array_equal(gs[k], os_[k], err_msg=f"{ctx} state[{k}]")
    np.testing.assert_array_equal(gs["contact_count"], os_["contact_count"], err_msg=f"{ctx} contact_count")
    for e in range(gs["contact_count"].shape[0]):
        n = int(gs["contact_count"][e])
        np.testing.assert_array_equal(gs["contact_ab"][e, :n], os_["contact_ab"][e, :n],
                                      err_msg=f"{ctx} env {e} contact order")
        np.testing.assert_array_equal(gs["contact_imp"][e, :n], os_["contact_imp"][e, :n],
                                      err_msg=f"{ctx} env {e} impulses")


def f32_obs_mismatch(gpu_obs, oracle_obs64):
    """Count float32 obs entries differing from the oracle's f64 obs rounded to f32."""
    ref = oracle_obs64.astype(np.float32)
    d = gpu_obs != ref
    if not d.any():
        return 0
    # tolerate 1-ulp differences (double atan2/cos/sin of ocml vs glibc round differently
    # in rare cases); anything else is a real mismatch
    ulp = np.abs(gpu_obs.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    bad = d & (ulp > 1)
    # angle wrap at exactly +-pi may flip sign: compare modulo 2pi
    if bad.any():
        diff = np.abs(((gpu_obs.astype(np.float64) - ref + np.pi) % (2 * np.pi)) - np.pi)
        bad &= diff > 1e-6
    assert not bad.any(), f"{int(bad.sum())} obs entries off by more than 1 ulp"
    return int(d.sum())


def oracle_for(cfg, tidx, E, seed, env_offset=0):
    return OracleFlock(cfg, tidx, E, seed, env_offset)


def combat_bot(obs, mask):
    """The reference's scripted TDM actor (test_scripts/bots.py:3-16), vectorised over
    the fixed-slot obs [E, N, N-1, 4] (r, t, p, is_ally) + mask: attack the closest
    enemy (first minimal r in list order), turning toward it, walking forward when
    it is within pi/5, attacking when r < 3; idle without enemies. Rows of dead
    agents are idle (they are not stepped)."""
    E, N = obs.shape[0], obs.shape[1]
    enemy = mask.astype(bool) & (obs[..., 3] == 0)
    r = np.where(enemy, obs[..., 0], np.inf)
    k = np.argmin(r, axis=-1)  # first index of the minimum == strict '<' scan
    has = enemy.any(axis=-1)
    sel = np.take_along_axis(obs, k[..., None, None].repeat(4, -1), axis=2)[..., 0, :]
    a = np.ones((E, N, 4), np.uint8)
    a[..., 3] = 0
    t = sel[..., 1]
    a[..., 0] = np.where(has, (np.abs(t) < np.pi / 5).astype(np.uint8) + 1, 1)
    a[..., 2] = np.where(has, (np.sign(t) + 1).astype(np.uint8), 1)
    a[..., 3] = np.where(has, (sel[..., 0] < 3).astype(np.uint8), 0)
    return a


def combat_bot_dict(obs):
    """bots.combat (test_scripts/bots.py:3-16) on one agent's reference-format obs
    dict, for driving the drop-in TDM through its `actors` hook."""
    enemies = [a for a in obs["agents"] if a["type"] == 0]
    if not enemies:
        return np.array([1, 1, 1, 0])
    closest = enemies[0]
    for a in enemies:
        if a["position"][0] < closest["position"][0]:
            closest = a
    rotation = np.sign(closest["position"][1]) + 1
    forward = int(np.abs(closest["position"][1]) < (np.pi / 5)) + 1
    attack = int(closest["position"][0] < 3)
    return np.array([forward, 1, rotation, attack])


def flock_bot(obs):
    """bots.flock (test_scripts/bots.py:37-61), vectorised over Flock obs [..., 4|6]:
    idle within r < 1 of the target, else turn toward it (sign(t) + 1) and walk
    forward when |t| < pi/4 (cartesian: sign(sin t) + 1, forward when cos t > cos(pi/4))."""
    od = obs.shape[-1]
    h = od // 2
    r = obs[..., h]
    a = np.ones(obs.shape[:-1] + (3,), np.uint8)
    if od == 6:
        rot = np.sign(obs[..., h + 2]) + 1
        fwd = (obs[..., h + 1] > np.cos(np.pi / 4)).astype(np.uint8) + 1
    else:
        rot = np.sign(obs[..., h + 1]) + 1
        fwd = (np.abs(obs[..., h + 1]) < (np.pi / 4)).astype(np.uint8) + 1
    far = ~(r < 1)
    a[..., 0] = np.where(far, fwd, 1)
    a[..., 2] = np.where(far, rot.astype(np.uint8), 1)
    return a
