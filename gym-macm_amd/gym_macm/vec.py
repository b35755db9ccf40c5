"""FlockVec — the batched throughput API for cm-flock-v0.

E independent Flock envs (reference gym_macm/envs/mvmnt.py) stepped by one HIP
launch per step, with actions and outputs as device tensors:

    env = FlockVec(num_envs=4096, n_agents=[64], seed=0)
    obs, nbr_id = env.obs, env.nbr_id            # initial observation
    obs, nbr_id, reward, done = env.step(actions)  # actions uint8 [E, N, 3] on the GPU

Env e is the reference env constructed after ``random.seed(seed + env_offset + e)``;
each env keeps that stream on the device, so ``reset_envs(mask)`` / ``autoreset=True``
start new episodes exactly as the env's own ``reset()`` would draw them.
shard a job over GPUs by giving each rank its contiguous ``env_offset``.
Settings keyword arguments are the reference's (flockSettings, settings.py:110-146).
Returned tensors are views of buffers reused by the next call.
"""
from __future__ import annotations

import numpy as np
import torch

from gym_macm.settings import flockSettings, to_config
from gym_macm.world import World


class FlockVec(object):
    def __init__(self, num_envs, n_agents=(10,), targets=None, seed=0, env_offset=0, device=None,
                 obs_dtype=torch.float32, max_contacts=0, autoreset=False, validate_actions=False, **kwargs):
        self.settings = flockSettings(**kwargs)
        self.num_envs = int(num_envs)
        self.n_agents = list(n_agents) if not isinstance(n_agents, int) else [n_agents]
        N = int(sum(self.n_agents))
        self.n_targets = 1 if targets is None else len(np.unique(targets))
        self.targets_idx = np.zeros(N, np.int32) if targets is None else np.asarray(targets, np.int32)
        cfg = to_config(self.settings, N, self.n_targets, obs_f64=(obs_dtype == torch.float64),
                        validate_actions=validate_actions)
        self.world = World(cfg, self.targets_idx, self.num_envs, device=device, max_contacts=max_contacts)
        self.device = self.world.device
        self.N = N
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self.autoreset = bool(autoreset)
        self.obs, self.nbr_id = self.world.reset(self.seed, self.env_offset)

    @property
    def obs_dim(self):
        return self.world.OD

    def reset(self, seed=None):
        if seed is not None:
            self.seed = int(seed)
        self.obs, self.nbr_id = self.world.reset(self.seed, self.env_offset)
        return self.obs, self.nbr_id

    def step(self, actions):
        """One step of every env. With ``autoreset``, envs whose episode ended in this
        step start their next episode right away (reset_envs on the done flags, on
        the device): the returned done marks them and obs already holds the new
        episode's initial observation for those envs.

        Raises MacmOverflowError (a MacmLibraryError) once an earlier step has overflowed a
        capacity (the contact list's max_contacts; dense touching contacts never overflow: the
        spill step takes them) — on the first call after the device reported it, which without a
        synchronisation may be a few queued steps later (check_status() is exact) —
        MacmInvalidActionError with ``validate_actions=True`` and an
        action outside the action space (no env is stepped, as the reference asserts first)."""
        out = self.world.step(actions)
        if self.autoreset:
            self.world.reset_envs(self.world.done)
        return out

    def rollout(self, actions, trajectory=False, traj=None):
        """K steps of every env with actions given in advance ([K, E, N, 3] on the device, e.g. a
        random-action rollout), one launch (World.rollout): each env runs its K steps back to back.
        Same results as K step() calls without autoreset; returns the last step's outputs, or with
        ``trajectory=True`` every step's (World.rollout_traj: a dict of [K, ...] tensors, written
        into ``traj`` if given). With ``autoreset`` a step-by-step loop is required."""
        if self.autoreset:
            raise ValueError("rollout steps without autoreset; use step() with autoreset=True")
        if trajectory:
            return self.world.rollout_traj(actions, traj)
        return self.world.rollout(actions)

    def rollout_bots(self, actions, n_steps, trajectory=False, traj=None):
        """n_steps of the closed loop step -> bots.flock -> step in one launch (World.rollout_bots);
        ``actions`` (uint8 [E, N, 3]) holds the first step's actions on entry, the next on return.
        ``trajectory=True``: actions is [n_steps + 1, E, N, 3] and every step's outputs and actions
        are kept (World.rollout_bots_traj)."""
        if self.autoreset:
            raise ValueError("rollout_bots steps without autoreset; use step() with autoreset=True")
        if trajectory:
            return self.world.rollout_bots_traj(actions, n_steps, traj)
        return self.world.rollout_bots(actions, n_steps)

    def reset_envs(self, mask=None):
        """New episodes in the masked envs (see World.reset_envs)."""
        return self.world.reset_envs(mask)

    def observe(self):
        return self.world.observe()

    def get_state(self):
        return self.world.get_state()

    def set_state(self, state):
        self.world.set_state(state)

    def status(self):
        return self.world.status()

    def check_status(self):
        """Raise MacmOverflowError if any env overflowed a capacity (synchronises)."""
        self.world.check_status()

    def spilled(self):
        """Env-steps taken by the spill step (dense envs) since creation."""
        return self.world.spilled()

    def counters(self):
        return self.world.counters()

    def reward_sums(self):
        """(per-env reward totals [E] float64, their sum in env order); World.reward_sums."""
        return self.world.reward_sums()
