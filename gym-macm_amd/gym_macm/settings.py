"""Settings mirror of the reference (gym_macm/settings.py).

``fwSettings`` (reference settings.py:25-59) and ``flockSettings``
(settings.py:110-146) keep the reference's attribute names and defaults so
``gym.make('gym_macm:cm-flock-v0', **kwargs)`` accepts the same keyword
arguments. GUI-only attributes (draw flags, checkboxes, sliders, the unused
argparse parser at settings.py:62-106) are kept as inert attributes only where a
user could plausibly read them. ``to_config`` flattens a settings object into the
C-ABI ``macm_config`` (include/macm.h).
"""
from __future__ import annotations

import numpy as np

from . import _abi


class CircleFixture:
    """Stand-in for the b2FixtureDef(shape=b2CircleShape(radius), density, friction)
    the reference stores in ``bodySettings['fixtures']`` (settings.py:127-132)."""

    def __init__(self, radius=0.5, density=1.0, friction=0.3):
        self.radius = radius
        self.density = density
        self.friction = friction


class fwSettings(object):
    # reference settings.py:25-59
    backend = 'pyglet'
    hz = 60.0
    velocityIterations = 8
    positionIterations = 3
    enableWarmStarting = True
    enableContinuous = True
    enableSubStepping = False
    drawStats = False
    drawShapes = True
    drawJoints = True
    drawCoreShapes = False
    drawAABBs = False
    drawOBBs = False
    drawPairs = False
    drawContactPoints = False
    maxContactPoints = 100
    drawContactNormals = False
    drawFPS = False
    drawMenu = True
    drawCOMs = False
    pointSize = 2.5
    pause = False
    singleStep = False
    onlyInit = False


class flockSettings(fwSettings):
    """reference settings.py:110-146 (kwargs are setattr'd, then reward_radius is derived)."""

    def __init__(self, **kwargs):
        super().__init__()
        self.render = False
        self.record = False
        self.record_dir = "../imgs/"
        self.verbose_display = True
        self.start_spread = 20
        self.start_point = [0, 0]
        self.agent_rotation_speed = 0.8 * (2 * np.pi)
        self.agent_force = 20
        self.time_limit = 60
        self.bodySettings = {"fixtures": CircleFixture(0.5, 1, 0.3), "linearDamping": 5,
                             "fixedRotation": True}
        self.action_mode = "discrete"
        self.reward_mode = "binary"
        self._reward_radius = 7
        self.target_mindist = 25
        self.target_maxdist = 60
        self.coord = "polar"
        for kw in kwargs:
            setattr(self, kw, kwargs[kw])
        self.reward_radius = self._reward_radius if self.reward_mode == "binary" else 1


def to_config(s: fwSettings, n_agents: int, n_targets: int, obs_f64: bool = False,
              validate_actions: bool = False) -> _abi.MacmConfig:
    """Flatten a settings object into ``macm_config``; rejects what the HIP path does not model."""
    if getattr(s, "render", False):
        raise NotImplementedError("render=True (pyglet GUI) is out of scope: headless NoRender only")
    # enableContinuous only gates SolveTOI, a no-op for all-dynamic non-bullet
    # worlds; sub-stepping would change the step itself.
    if getattr(s, "enableSubStepping", False):
        raise NotImplementedError("enableSubStepping=True is not modelled")
    if s.action_mode not in ("discrete", "continuous"):
        raise ValueError(f"action_mode {s.action_mode!r}")
    if s.reward_mode not in ("binary", "linear"):
        raise ValueError(f"reward_mode {s.reward_mode!r}")
    if s.coord not in ("polar", "cartesian"):
        raise ValueError(f"coord {s.coord!r}")
    fx = s.bodySettings.get("fixtures")
    if not bool(s.bodySettings.get("fixedRotation", False)):
        raise NotImplementedError("fixedRotation=False is not modelled (reference default is True)")
    c = _abi.MacmConfig()
    c.n_agents = int(n_agents)
    c.n_targets = int(n_targets)
    c.action_mode = _abi.ACTION_DISCRETE if s.action_mode == "discrete" else _abi.ACTION_CONTINUOUS
    c.reward_mode = _abi.REWARD_BINARY if s.reward_mode == "binary" else _abi.REWARD_LINEAR
    c.coord = _abi.COORD_POLAR if s.coord == "polar" else _abi.COORD_CARTESIAN
    c.velocity_iterations = int(s.velocityIterations)
    c.position_iterations = int(s.positionIterations)
    c.warm_starting = 1 if s.enableWarmStarting else 0
    c.obs_f64 = 1 if obs_f64 else 0
    c.validate_actions = 1 if validate_actions else 0
    c.hz = float(s.hz)
    c.start_spread = float(s.start_spread)
    c.start_point[0] = float(s.start_point[0])
    c.start_point[1] = float(s.start_point[1])
    c.agent_rotation_speed = float(s.agent_rotation_speed)
    c.agent_force = float(s.agent_force)
    c.time_limit = float(s.time_limit)
    c.reward_radius = float(s.reward_radius)
    c.target_mindist = float(s.target_mindist)
    c.target_maxdist = float(s.target_maxdist)
    c.radius = float(getattr(fx, "radius", 0.5))
    c.density = float(getattr(fx, "density", 1.0))
    c.friction = float(getattr(fx, "friction", 0.3))
    c.linear_damping = float(s.bodySettings.get("linearDamping", 0.0))
    return c


class combatSettings(fwSettings):
    """reference settings.py:149-177. The reference ignores kwargs here; like
    flockSettings they are applied."""

    def __init__(self, **kwargs):
        super().__init__()
        self.render = False
        self.record = False
        self.record_dir = "../imgs/"
        self.verbose_display = True
        self.start_spread = 20
        self.start_point = [0, 0]
        self.agent_rotation_speed = 0.8 * (2 * np.pi)
        self.agent_force = 20
        self.time_limit = 60
        self.cooldown_atk = 1
        self.cooldown_mov_penalty = 0.5
        self.bodySettings = {"fixtures": CircleFixture(0.5, 1, 0.3), "linearDamping": 5,
                             "fixedRotation": True}
        for kw in kwargs:
            setattr(self, kw, kwargs[kw])


def to_tdm_config(s: combatSettings, n_agents, obs_f64=False, fresh_raycast=False, decay_mov_penalty=False,
                  world_width=30.0, world_height=30.0, validate_actions=False):
    """Flatten combatSettings + TDM/Agent constants (combat.py:13-29,76-77) into macm_tdm_config."""
    sizes = [int(n) for n in n_agents]
    if not 1 <= len(sizes) <= 4:
        raise ValueError("TDM supports 1 to 4 teams")
    c = _abi.tdm_config_from_defaults()
    c.n_teams = len(sizes)
    for t in range(4):
        c.team_size[t] = sizes[t] if t < len(sizes) else 0
    c.n_agents = sum(sizes)
    c.velocity_iterations = int(s.velocityIterations)
    c.position_iterations = int(s.positionIterations)
    c.warm_starting = 1 if s.enableWarmStarting else 0
    c.obs_f64 = 1 if obs_f64 else 0
    c.validate_actions = 1 if validate_actions else 0
    c.fresh_raycast = 1 if fresh_raycast else 0
    c.decay_mov_penalty = 1 if decay_mov_penalty else 0
    c.hz = float(s.hz)
    c.world_width = float(world_width)
    c.world_height = float(world_height)
    c.agent_rotation_speed = float(s.agent_rotation_speed)
    c.agent_force = float(s.agent_force)
    c.time_limit = float(s.time_limit)
    c.cooldown_atk = float(s.cooldown_atk)
    c.cooldown_mov_penalty = float(s.cooldown_mov_penalty)
    fx = s.bodySettings["fixtures"]
    c.radius, c.density, c.friction = float(fx.radius), float(fx.density), float(fx.friction)
    c.linear_damping = float(s.bodySettings["linearDamping"])
    return c
