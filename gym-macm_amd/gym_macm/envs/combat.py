"""Drop-in ``TDM`` env (reference gym_macm/envs/combat.py:57-264) over the HIP world.

Same constructor, attributes (agents with string ids ``str(team) + str(j)``,
health / alive / cooldowns, ``n_alive``, ``done``, ``winner``, ``time_passed``)
and ``step(actions) -> obs`` dict surface as the reference; the per-agent loops
(rotation / force / melee :121-155, deaths :157-165, Box2D step :167, get_obs
:206-227) run as one HIP launch over an E=1 world (gym_macm.tdm_world). Spawn
poses come from Python's global ``random`` in the reference's order (:80-85), so
``random.seed(s); TDM(...)`` reproduces the reference env for seed s.

The reference cannot be constructed as shipped (:65 uses ``combatSettings``,
which :8 never imports; :150-151 and :173 read ``self.cooldown_atk``,
``self.cooldown_mov_penalty``, ``self.time_limit``, which are never set). This
env supplies those four names from combatSettings and is otherwise literal,
including the shared never-reset ray-cast listener and the never-decremented
movement penalty; ``fresh_raycast=True`` / ``decay_mov_penalty=True`` switch
those off (DESIGN.md "TDM"). Documented differences: ``render`` must be falsy
(headless only; the reference's default is the truthy string "False"), and
``reset()`` revives every agent (the reference's leaves dead bodies inactive,
:234-245).

``ControlledTDM`` (keyboard/mouse-controlled, :266-358) is out of scope.
"""
from __future__ import annotations

import random

import numpy as np
import torch

from gym_macm import spaces
from gym_macm.envs.mvmnt import Color, Vec2
from gym_macm.settings import combatSettings, to_tdm_config
from gym_macm.tdm_world import TdmWorld


class _BodyView(object):
    """Read-only view of an agent's body (position, angle, linearVelocity, active)."""

    def __init__(self, env, i):
        self._env = env
        self._i = i

    @property
    def position(self):
        return Vec2(*self._env._host_state()["pos"][0, self._i])

    @property
    def angle(self):
        return float(self._env._host_state()["angle"][0, self._i])

    @property
    def linearVelocity(self):
        return Vec2(*self._env._host_state()["vel"][0, self._i])

    @property
    def active(self):
        return bool(self._env._host_state()["alive"][0, self._i])


class Agent(object):
    """reference combat.py:13-54; health and alive mirror the device state after every
    step, the cooldowns are read from it on access."""

    def __init__(self, ID, team=0, actor=None, env=None, index=0):
        self._env = env
        self._k = index
        self.init_health = 1
        self.team = team
        self.id = ID
        self.actor = actor
        self.rotation_speed = 0.8 * (2 * np.pi)
        self._force = 20
        self.melee_range = 2
        self.melee_dmg = 0.25
        self.percent_mov_penalty = 0.2
        self.health = self.init_health
        self.alive = True
        self.body = None

    @property
    def cooldown_atk(self):
        return float(self._env._host_state()["cd_atk"][0, self._k]) if self._env else 0

    @property
    def cooldown_mov_penalty(self):
        return float(self._env._host_state()["cd_mov"][0, self._k]) if self._env else 0

    @property
    def color(self):
        if hasattr(self, "_color"):
            return self._color
        return {0: Color(0.2, 0.2, 1), 1: Color(1, 0.2, 0.2), 2: Color(0.2, 1, 0.2)}.get(self.team)

    @property
    def force(self):
        return self._force * (1 - self.percent_mov_penalty * int(self.cooldown_mov_penalty > 0))


class TDM(object):
    name = "Team Deathmatch"
    description = "TDM on an empty world"

    def __init__(self, render=False, n_agents=[1, 1], actors=None, colors=None, device=None,
                 fresh_raycast=False, decay_mov_penalty=False, **kwargs):
        if render and render != "False":
            raise NotImplementedError("render=True (pyglet) is out of scope; headless only")
        self.settings = combatSettings(**kwargs)
        self.done = False
        self.winner = None
        self.n_agents = list(n_agents)
        self.world_width = 30
        self.world_height = 30
        self.time_passed = 0
        self.cooldown_atk = self.settings.cooldown_atk
        self.cooldown_mov_penalty = self.settings.cooldown_mov_penalty
        self.time_limit = self.settings.time_limit
        self.agents = []
        N = int(sum(self.n_agents))
        self._N = N
        pos, ang = self._draw_poses()
        for i in range(len(self.n_agents)):
            for j in range(self.n_agents[i]):
                agent = Agent(team=i, ID=str(i) + str(j), env=self, index=len(self.agents))
                if actors:
                    agent.actor = actors[i][j]
                if colors:
                    agent._color = colors[i]
                agent.body = _BodyView(self, len(self.agents))
                self.agents.append(agent)
        cfg = to_tdm_config(self.settings, self.n_agents, obs_f64=True, fresh_raycast=fresh_raycast,
                            decay_mov_penalty=decay_mov_penalty, world_width=self.world_width,
                            world_height=self.world_height)
        # one env: outputs and actions in pinned host memory (zero-copy views)
        self.world = TdmWorld(cfg, 1, device=device, host_outputs=True)
        self._act = torch.ones((1, N, 4), dtype=torch.uint8, pin_memory=True)
        self._act_np = self._act.numpy()
        self._cache = None
        self.world.place(pos[None], ang[None])
        self.n_alive = self.n_agents.copy()
        self.create_space()
        self.create_space_flag = False
        self.obs = self._obs_dict()

    # -- helpers --------------------------------------------------------------
    def _draw_poses(self):
        """combat.py:80-85 draw order: per agent in team order x, y, angle."""
        pos = np.zeros((self._N, 2), np.float32)
        ang = np.zeros((self._N,), np.float32)
        k = 0
        for i in range(len(self.n_agents)):
            for _ in range(self.n_agents[i]):
                x = random.random() * (i + self.world_width / 2)
                y = random.random() * self.world_height
                pos[k] = (x, y)
                ang[k] = random.uniform(-1, 1) * np.pi
                k += 1
        return pos, ang

    def _host_state(self):
        if self._cache is None:
            self._cache = self.world.get_state()
        return self._cache

    def _sync(self):
        torch.cuda.current_stream(self.world.device).synchronize()

    def _sync_agents(self):
        health = self.world.health[0].numpy()
        alive = self.world.alive[0].numpy()
        for k, agent in enumerate(self.agents):
            agent.health = float(health[k])
            agent.alive = bool(alive[k])

    def _obs_dict(self):
        obs = self.world.obs[0].numpy()  # pinned host outputs: views, copied per entry below
        mask = self.world.mask[0].numpy()
        self._sync_agents()
        out = {}
        N = self._N
        for i, agent in enumerate(self.agents):
            if not agent.alive:
                continue
            others = []
            for k in range(N - 1):
                if mask[i, k]:
                    r, t, p, ally = obs[i, k]
                    others.append({"type": int(ally), "position": np.array([r, t, p])})
            out[agent.id] = {"myHealth": np.array([agent.health]), "myTeam": agent.team, "agents": others}
        return out

    # -- reference API ------------------------------------------------------------
    def step(self, actions=None):
        if self.done:  # combat.py:106-107: stepping continues after done
            self.quit()
        if actions is None:
            actions = {}
            for agent in self.agents:
                if not agent.alive:
                    continue
                actions[agent.id] = agent.actor(self.obs[agent.id])
        assert self.action_space.contains(actions)
        a = self._act_np
        for k, agent in enumerate(self.agents):
            a[0, k] = actions[agent.id] if agent.alive else (1, 1, 1, 0)
        self.world.step(self._act)
        self._sync()
        self.world.check_status()  # a TDM capacity overflow raises right here
        self._cache = None
        alive_before = [agent.alive for agent in self.agents]
        self.obs = self._obs_dict()
        died = False
        for agent, was in zip(self.agents, alive_before):
            if was and not agent.alive:
                self.n_alive[agent.team] -= 1
                died = True
        if died:
            self.create_space()
        self.time_passed += (1 / self.settings.hz)
        self.done = bool(self.world.done[0])
        w = int(self.world.winner[0])
        self.winner = None if w < 0 else w
        return self.obs

    def create_space(self):
        """combat.py:186-201"""
        alive = [agent for agent in self.agents if agent.alive]
        self.action_space = spaces.Dict({agent.id: spaces.MultiDiscrete([3, 3, 3, 2]) for agent in alive})
        self.observation_space = spaces.Dict(
            {agent.id: spaces.Dict({"myHealth": spaces.Box(np.array([0.0]), np.array([1.0])),
                                    "myTeam": spaces.Discrete(1),
                                    "agents": spaces.Tuple([spaces.Dict({
                                        "type": spaces.Discrete(1),
                                        "position": spaces.Box(np.array([0, -np.pi, -np.pi]),
                                                               np.array([np.inf, np.pi, np.pi]))})]
                                        * (len(alive) - 1))})
             for agent in alive})

    def get_rewards(self):
        """combat.py:203-204: TDM has no rewards."""
        pass

    def get_obs(self):
        self.world.observe()
        self._sync()
        return self._obs_dict()

    def reset(self):
        """New spawn poses from the global RNG (combat.py:234-245 draw order), every
        agent revived with full health and zero cooldowns."""
        self.done = False
        self.winner = None
        self.time_passed = 0
        pos, ang = self._draw_poses()
        self.world.place(pos[None], ang[None])
        self._cache = None
        self.n_alive = self.n_agents.copy()
        self.obs = self._obs_dict()
        self.create_space()
        return self.obs

    def run(self):
        pass

    def quit(self):
        pass


class ControlledTDM(TDM):
    """Human-controlled TDM (combat.py:266-358: keyboard/mouse through pyglet) — out of scope."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("cm-ctdm-v0 is human-controlled (keyboard/mouse, pyglet); out of scope")
