"""Drop-in ``Flock`` env (reference gym_macm/envs/mvmnt.py:27-272) over the HIP world.

Same constructor, attributes and ``step(actions) -> (obs, rewards)`` dict surface
as the reference; the per-agent Python loops (action->force :97-129, Box2D step
through FrameworkBase :131, get_rewards :160-179, get_obs :181-222) run as one
HIP launch over an E=1 world (gym_macm.world.World). Initial poses are drawn from
Python's global ``random`` module in the reference's order (:47-64), so
``random.seed(s); Flock(...)`` reproduces the reference env for seed s and leaves
the global RNG in the same state.

Observations are computed in float64 on the GPU (config obs_f64); rewards are the
reference's Python types (int -1/0/1 in binary mode, float in linear mode).
The rewards dict keeps the reference's insertion order (:160-179): the two agents of
every contact in ``world.contacts`` order first (fixture A, then B), then the others
in ascending id (``reward_key_order``). Documented difference: ``reset()`` works (the
reference's raises AttributeError, :224-233).
"""
from __future__ import annotations

import random

import numpy as np
import torch

from gym_macm import spaces
from gym_macm.settings import flockSettings, to_config
from gym_macm.world import World


def reward_key_order(prev_ab, next_ab, n_agents):
    """The key order of the reference's rewards dict after a step (mvmnt.py:160-179): -1 goes in
    for ``contact.fixtureA`` then ``contact.fixtureB`` of every contact in ``world.contacts`` order,
    then every other agent in ascending id.

    ``world.contacts`` at that point is Box2D's list after the step: the contacts created by the
    step's closing FindNewContacts, prepended (``b2ContactManager::AddPair``), ahead of the contacts
    that survived the step's Collide in their order. The world keeps an ordered list per env of the
    contacts that survive the NEXT Collide (entries a | b << 16, fixture A in the low half): before the
    step (``prev_ab``) that is exactly what the step's Collide keeps; after it (``next_ab``) it is the
    new contacts ahead of the survivors that still overlap. So ``world.contacts`` = the entries of
    ``next_ab`` absent from ``prev_ab``, in order, followed by ``prev_ab``."""
    prev = [int(x) for x in prev_ab]
    old = set(prev)
    order = dict()
    for x in [int(x) for x in next_ab if int(x) not in old] + prev:
        order.setdefault(x & 0xFFFF, None)
        order.setdefault(x >> 16, None)
    n_contact = len(order)
    for i in range(n_agents):
        order.setdefault(i, None)
    return list(order), n_contact


class Color(object):
    """Stand-in for b2Color (render-only attribute of Agent)."""

    def __init__(self, r, g, b):
        self.r, self.g, self.b = r, g, b


class Vec2(object):
    """Read-only float32 2-vector with b2Vec2-like access (x, y, [i])."""

    __slots__ = ("x", "y")

    def __init__(self, x, y):
        self.x = float(np.float32(x))
        self.y = float(np.float32(y))

    def __getitem__(self, i):
        return (self.x, self.y)[i]

    def __iter__(self):
        return iter((self.x, self.y))

    def __len__(self):
        return 2

    def __repr__(self):
        return "Vec2(%r, %r)" % (self.x, self.y)


class _BodyView(object):
    """Read-only view of an agent's body state (position, angle, velocity)."""

    def __init__(self, env, i):
        self._env = env
        self._i = i

    @property
    def position(self):
        s = self._env._host_state()
        return Vec2(*s["pos"][0, self._i])

    @property
    def angle(self):
        return float(self._env._host_state()["angle"][0, self._i])

    @property
    def linearVelocity(self):
        s = self._env._host_state()
        return Vec2(*s["vel"][0, self._i])


class Agent(object):
    """reference mvmnt.py:15-25"""

    def __init__(self, settings, ID, actor=None):
        self.id = ID
        self.actor = actor
        self.rotation_speed = settings.agent_rotation_speed
        self.force = settings.agent_force
        self._color = Color(0.4, 0.4, 0.6)
        self.color = Color(0.4, 0.4, 0.6)
        self.body = None

    def reset_color(self):
        self.color = self._color


class Flock(object):
    name = "Flock v0"
    description = "Flock"

    def __init__(self, n_agents=[10], actors=None, colors=None, targets=None, device=None, **kwargs):
        self.settings = flockSettings(**kwargs)
        s = self.settings
        if s.render:
            raise NotImplementedError("render=True (pyglet) is out of scope; headless only")
        self.done = False
        self.n_agents = n_agents
        N = int(sum(n_agents))
        self.n_targets = 1 if targets is None else len(np.unique(targets))
        # the reference defaults to [0] * n_agents[0] (mvmnt.py:43), which only covers
        # single-flock n_agents; [0] * N is identical there and also valid for lists.
        self.targets_idx = [0] * N if targets is None else list(targets)
        self.time_passed = 0
        # mvmnt.py:46-52: target poses from the global RNG
        tg = np.zeros((self.n_targets, 2), np.float32)
        for t in range(self.n_targets):
            self.t_min, self.t_max = s.target_mindist, s.target_maxdist
            rand_angle = 2 * np.pi * random.random()
            rand_dist = self.t_min + random.random() * (self.t_max - self.t_min)
            tg[t] = (rand_dist * np.cos(rand_angle), rand_dist * np.sin(rand_angle))
        # mvmnt.py:60-76: agent poses
        pos = np.zeros((N, 2), np.float32)
        ang = np.zeros((N,), np.float32)
        self.agents = []
        for i in range(N):
            x = s.start_spread * (random.random() - 0.5) + s.start_point[0]
            y = s.start_spread * (random.random() - 0.5) + s.start_point[1]
            angle = random.uniform(-1, 1) * np.pi
            pos[i] = (x, y)
            ang[i] = angle
            agent = Agent(s, ID=i)
            if actors:
                agent.actor = actors[i]
            if colors:
                agent._color = colors[i]
            agent.body = _BodyView(self, i)
            self.agents.append(agent)
        self.targets = [Vec2(*tg[t]) for t in range(self.n_targets)]
        cfg = to_config(s, N, self.n_targets, obs_f64=True)
        # one env: outputs (and actions) in pinned host memory, read as zero-copy views
        self.world = World(cfg, np.asarray(self.targets_idx, np.int32), 1, device=device, host_outputs=True)
        if s.action_mode == "discrete":
            self._act = torch.ones((1, N, 3), dtype=torch.uint8, pin_memory=True)
        else:
            self._act = torch.zeros((1, N, 2), dtype=torch.float32, pin_memory=True)
        self._act_np = self._act.numpy()
        self._N = N
        self._cache = None
        obs, nbr = self.world.place(pos[None], ang[None], tg[None])
        self._ab = self.world.contact_list(0)  # world.contacts order as of the next step's start
        self.create_space()
        self.create_space_flag = False
        self.obs = self._obs_dict(obs, nbr)

    # -- helpers --------------------------------------------------------------
    def _host_state(self):
        if self._cache is None:
            self._cache = self.world.get_state()
        return self._cache

    def _sync(self):
        torch.cuda.current_stream(self.world.device).synchronize()

    def _obs_dict(self, obs_t, nbr_t):
        obs = obs_t[0].numpy()  # pinned host output: a view, copied per node below
        nbr = nbr_t[0].numpy()
        N = self._N
        half = obs.shape[1] // 2
        out = {}
        for agent in self.agents:
            i = agent.id
            out[i] = {"nodes": [
                {"type": 0, "id": int(nbr[i]), "position": obs[i, :half].copy()},
                {"type": 1, "id": N, "position": obs[i, half:].copy()},
            ]}
        return out

    # -- reference API -----------------------------------------------------------
    def step(self, actions=None):
        if self.done:  # mvmnt.py:83-84: stepping continues after done
            self.quit()
        if actions is None:
            actions = {}
            for agent in self.agents:
                actions[agent.id] = agent.actor({agent.id: self.obs[agent.id]})
        assert self.action_space.contains(actions)
        a = self._act_np
        for agent in self.agents:
            a[0, agent.id] = actions[agent.id]
        obs_t, nbr_t, rew_t, _ = self.world.step(self._act)
        self._sync()
        self._cache = None
        # the dict API waits for every step anyway: a capacity overflow (only the contact list
        # can overflow; dense touching contacts take the spill step) raises right here
        self.world.check_status()
        obs = obs_t[0].numpy()
        rew = rew_t[0].numpy()
        half = obs.shape[1] // 2
        nxt = self.world.contact_list(0)
        keys, n_contact = reward_key_order(self._ab, nxt, self._N)
        self._ab = nxt
        if n_contact != int((rew == -1.0).sum()) or any(rew[i] != -1.0 for i in keys[:n_contact]):
            raise RuntimeError("the contact list and the step's -1 rewards disagree (a capacity overflowed?)")
        rewards = {}
        for i in keys:
            if rew[i] == -1.0:
                rewards[i] = -1
            elif self.settings.reward_mode == "linear":
                d = obs[i, half]  # target node r == sqrt(b2DistanceSquared(target, position))
                rewards[i] = (-d / 35) + 1
            else:
                rewards[i] = int(rew[i])
        self.time_passed += (1 / self.settings.hz)
        if self.time_passed > self.settings.time_limit:
            self.done = True
        self.obs = self._obs_dict(obs_t, nbr_t)
        return self.obs, rewards

    def create_space(self):
        """mvmnt.py:142-158 (the declared obs space lists N+1 nodes; get_obs emits 2)."""
        if self.settings.action_mode == "discrete":
            self.action_space = spaces.Dict({agent.id: spaces.MultiDiscrete([3, 3, 3]) for agent in self.agents})
        if self.settings.action_mode == "continuous":
            self.action_space = spaces.Dict({agent.id: spaces.Box(np.array([-1, -1]), np.array([1, 1]))
                                             for agent in self.agents})
        self.observation_space = spaces.Dict(
            {agent.id: spaces.Dict({"nodes": spaces.Tuple([spaces.Dict({
                "type": spaces.Discrete(1), "id": spaces.Discrete(1),
                "position": spaces.Box(np.array([0, -np.pi]), np.array([np.inf, np.pi]))})] * (len(self.agents) + 1))})
             for agent in self.agents})

    def get_obs(self):
        obs, nbr = self.world.observe()
        self._sync()
        return self._obs_dict(obs, nbr)

    def reset(self):
        """Working reset (the reference's raises AttributeError, mvmnt.py:224-233): new
        agent poses from the global RNG (same draw order as __init__), targets kept."""
        s = self.settings
        self.done = False
        self.time_passed = 0
        pos = np.zeros((self._N, 2), np.float32)
        ang = np.zeros((self._N,), np.float32)
        for i in range(self._N):
            x = s.start_spread * (random.random() - 0.5) + s.start_point[0]
            y = s.start_spread * (random.random() - 0.5) + s.start_point[1]
            ang[i] = random.uniform(-1, 1) * np.pi
            pos[i] = (x, y)
        tg = np.array([[t.x, t.y] for t in self.targets], np.float32)
        obs, nbr = self.world.place(pos[None], ang[None], tg[None])
        self._ab = self.world.contact_list(0)
        self._cache = None
        self.create_space()
        self.obs = self._obs_dict(obs, nbr)
        return self.obs

    def run(self):
        """NoRender.run is a no-op (no_render.py:13-14)."""
        pass

    def quit(self):
        pass

    def BeginContact(self, agent1, agent2):
        pass
