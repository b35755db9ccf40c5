"""Generate golden vectors by running the REFERENCE's own env code.

Run in the build container only (needs /root/reference; never on the GPU box):
    python tests/golden/make_golden.py

It imports gym_macm/envs/mvmnt.py (Flock) and test_scripts/bots.py from
/root/reference unmodified, with two stand-ins for absent third-party packages:
  * tests/golden/gym_stub.py      — `gym` (Env base, spaces, register)
  * tests/golden/box2d_facade.py  — `Box2D`, backed by the oracle's b2lite world
Each scenario seeds the stdlib `random` (which the reference uses for targets,
positions and angles, mvmnt.py:49-64), builds Flock(...) and steps it with either
seeded random actions or the reference's bots.flock actors (actor mode,
mvmnt.py:86-92), recording the per-step observation dicts, reward dicts and done
flag as arrays in tests/golden/<name>.npz. What this pins: the env layer exactly
as the reference computes it. What it does not pin: Box2D's dynamics (the facade's
physics is the oracle's restatement; see DESIGN.md "Parity").
"""
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import box2d_facade  # noqa: E402
import gym_stub  # noqa: E402

SCENARIOS = [
    dict(name="c1_n4_random", seed=0, n_agents=[4], steps=200, policy="random"),
    dict(name="n4_bots", seed=7, n_agents=[4], steps=400, policy="bots"),
    dict(name="n8_bots_long", seed=5, n_agents=[8], steps=900, policy="bots"),
    dict(name="n16_multiflock_linear_cart", seed=3, n_agents=[16], targets=[0] * 8 + [1] * 8,
         kwargs=dict(reward_mode="linear", coord="cartesian"), steps=150, policy="random"),
    dict(name="n64_random", seed=11, n_agents=[64], steps=60, policy="random"),
    dict(name="n6_done_hz30", seed=2, n_agents=[6], kwargs=dict(hz=30.0, time_limit=1.0), steps=40,
         policy="random"),
    dict(name="n6_continuous", seed=4, n_agents=[6], kwargs=dict(action_mode="continuous"), steps=100,
         policy="random_cont"),
    dict(name="n12_split_3targets", seed=21, n_agents=[5, 7], targets=[0, 1, 2] * 4, steps=120,
         policy="bots"),
    # random actions with the target drawn 1-3 m from a dense start (start_spread 5): positive
    # binary rewards and collisions from the first step, without a scripted policy
    dict(name="n24_near_target_dense", seed=13, n_agents=[24],
         kwargs=dict(start_spread=5, target_mindist=1, target_maxdist=3), steps=150, policy="random"),
]

# TDM (combat.py). Stepped until done or `steps`.
TDM_SCENARIOS = [
    dict(name="tdm_2x4_bots", seed=1, n_agents=[4, 4], steps=900, policy="combat"),
    dict(name="tdm_2x8_random", seed=2, n_agents=[8, 8], steps=300, policy="random"),
    dict(name="tdm_3x3_bots", seed=3, n_agents=[3, 3, 3], steps=900, policy="combat"),
    dict(name="tdm_2x16_bots", seed=4, n_agents=[16, 16], steps=700, policy="combat"),
    dict(name="tdm_1x2_4x1_mixed", seed=5, n_agents=[2, 1, 1, 1], steps=600, policy="combat"),
]

TDM_NOTE = ("combat.py as shipped cannot run: it never imports combatSettings (:65) and reads "
            "self.cooldown_atk/.cooldown_mov_penalty/.time_limit (:150-151,:173) that are never set. "
            "This script supplies exactly those four names from gym_macm.settings.combatSettings at run "
            "time and changes nothing else.")


def flatten_obs(obs, N):
    nbr = np.zeros(N, np.int32)
    od = len(obs[0]["nodes"][0]["position"])
    pos = np.zeros((N, 2 * od), np.float64)
    for i in range(N):
        nodes = obs[i]["nodes"]
        assert len(nodes) == 2 and nodes[0]["type"] == 0 and nodes[1]["type"] == 1
        assert nodes[1]["id"] == N
        nbr[i] = nodes[0]["id"]
        pos[i, :od] = nodes[0]["position"]
        pos[i, od:] = nodes[1]["position"]
    return nbr, pos


def run(sc):
    from gym_macm.envs.mvmnt import Flock  # reference code
    import bots  # reference test_scripts/bots.py

    N = sum(sc["n_agents"])
    kw = dict(sc.get("kwargs", {}))
    rng = np.random.default_rng(1000 + sc["seed"])
    recorded = []
    actors = None
    if sc["policy"] == "bots":
        def make_actor():
            def actor(o):
                a = bots.flock(o)
                recorded.append(np.asarray(a))
                return a
            return actor
        actors = [make_actor() for _ in range(N)]
    random.seed(sc["seed"])
    env = Flock(n_agents=sc["n_agents"], actors=actors, targets=sc.get("targets"), **kw)
    T = len(env.targets)
    out = dict(
        targets=np.array([[t.x, t.y] for t in env.targets], np.float32),
        targets_idx=np.array(env.targets_idx, np.int32),
        init_pos=np.array([[a.body.position.x, a.body.position.y] for a in env.agents], np.float32),
        init_angle=np.array([np.float32(a.body.angle) for a in env.agents], np.float32),
    )
    out["init_nbr"], out["init_obs"] = flatten_obs(env.obs, N)
    S = sc["steps"]
    acts, nbrs, obss, rews, dones, poss, angs, orders, tps = [], [], [], [], [], [], [], [], []
    for t in range(S):
        if sc["policy"] == "random":
            a = rng.integers(0, 3, size=(N, 3))
            actions = {agent.id: a[agent.id] for agent in env.agents}
            obs, rewards = env.step(actions)
            acts.append(a.astype(np.uint8))
        elif sc["policy"] == "random_cont":
            a = rng.uniform(-1, 1, size=(N, 2)).astype(np.float32)
            actions = {agent.id: a[agent.id] for agent in env.agents}
            obs, rewards = env.step(actions)
            acts.append(a)
        else:
            recorded.clear()
            obs, rewards = env.step()
            a = np.stack(recorded).astype(np.uint8)
            assert a.shape == (N, 3)
            acts.append(a)
        nbr, pos = flatten_obs(obs, N)
        nbrs.append(nbr)
        obss.append(pos)
        rews.append(np.array([float(rewards[i]) for i in range(N)], np.float64))
        orders.append(np.array(list(rewards.keys()), np.int32))
        dones.append(bool(env.done))
        tps.append(env.time_passed)
        poss.append(np.array([[ag.body.position.x, ag.body.position.y] for ag in env.agents], np.float32))
        angs.append(np.array([np.float32(ag.body.angle) for ag in env.agents], np.float32))
    out.update(actions=np.stack(acts), nbr=np.stack(nbrs), obs=np.stack(obss), reward=np.stack(rews),
               reward_order=np.stack(orders), done=np.array(dones), time_passed=np.array(tps),
               pos=np.stack(poss), angle=np.stack(angs))
    s = env.settings
    meta = dict(name=sc["name"], seed=sc["seed"], n_agents=sc["n_agents"], N=N, T=T, steps=S,
                policy=sc["policy"], kwargs=kw, targets=sc.get("targets"),
                settings=dict(hz=s.hz, action_mode=s.action_mode, reward_mode=s.reward_mode,
                              coord=s.coord, reward_radius=s.reward_radius, time_limit=s.time_limit))
    out["meta"] = np.array(json.dumps(meta))
    return out


def tdm_slots(obs, agents, N):
    """obs dict -> fixed slots [N, N-1, 4] (r, t, p, type) + mask; slot k of agent i is
    agent j = k if k < i else k + 1 (the reference lists alive others in agent order)."""
    o = np.zeros((N, N - 1, 4), np.float64)
    m = np.zeros((N, N - 1), np.uint8)
    for i, ag in enumerate(agents):
        if ag.id not in obs:
            assert not ag.alive
            continue
        others = [j for j in range(N) if j != i and agents[j].alive]
        lst = obs[ag.id]["agents"]
        assert len(lst) == len(others)
        assert float(obs[ag.id]["myHealth"][0]) == ag.health and obs[ag.id]["myTeam"] == ag.team
        for j, d in zip(others, lst):
            k = j if j < i else j - 1
            o[i, k, :3] = d["position"]
            o[i, k, 3] = d["type"]
            m[i, k] = 1
    return o, m


def run_tdm(sc):
    import gym_macm.envs.combat as combat  # reference code
    from gym_macm.settings import combatSettings
    import bots

    combat.combatSettings = combatSettings          # missing import (combat.py:65)
    N = sum(sc["n_agents"])
    rng = np.random.default_rng(2000 + sc["seed"])
    recorded = {}
    actors = None
    if sc["policy"] == "combat":
        def make_actor(i):
            def actor(o):
                a = bots.combat(o)
                recorded[i] = np.asarray(a)
                return a
            return actor
        actors, i = [], 0
        for n in sc["n_agents"]:
            actors.append([make_actor(i + j) for j in range(n)])
            i += n
    random.seed(sc["seed"])
    env = combat.TDM(render=False, n_agents=list(sc["n_agents"]), actors=actors)
    st = env.settings
    env.cooldown_atk = st.cooldown_atk              # combat.py:150
    env.cooldown_mov_penalty = st.cooldown_mov_penalty  # :151
    env.time_limit = st.time_limit                  # :173
    ag = env.agents
    out = dict(team=np.array([a.team for a in ag], np.int32),
               init_pos=np.array([[a.body.position.x, a.body.position.y] for a in ag], np.float32),
               init_angle=np.array([np.float32(a.body.angle) for a in ag], np.float32))
    out["init_obs"], out["init_mask"] = tdm_slots(env.obs, ag, N)
    rec = {k: [] for k in ("actions", "obs", "mask", "health", "alive", "done", "winner", "pos", "angle",
                           "cd_atk", "cd_mov", "time_passed", "listener")}
    lst = env.framework.raycastListener
    for t in range(sc["steps"]):
        a = np.zeros((N, 4), np.uint8)
        if sc["policy"] == "random":
            r = np.concatenate([rng.integers(0, 3, size=(N, 3)), (rng.random((N, 1)) < 0.3)], axis=1)
            actions = {x.id: r[i] for i, x in enumerate(ag) if x.alive}
            for i, x in enumerate(ag):
                if x.alive:
                    a[i] = r[i]
            env.step(actions)
        else:
            recorded.clear()
            env.step()
            for i, v in recorded.items():
                a[i] = v
        rec["actions"].append(a)
        o, m = tdm_slots(env.obs, ag, N)
        rec["obs"].append(o)
        rec["mask"].append(m)
        rec["health"].append(np.array([x.health for x in ag], np.float64))
        rec["alive"].append(np.array([x.alive for x in ag], np.uint8))
        rec["done"].append(bool(env.done))
        rec["winner"].append(-1 if env.winner is None else int(env.winner))
        rec["pos"].append(np.array([[x.body.position.x, x.body.position.y] for x in ag], np.float32))
        rec["angle"].append(np.array([np.float32(x.body.angle) for x in ag], np.float32))
        rec["cd_atk"].append(np.array([x.cooldown_atk for x in ag], np.float64))
        rec["cd_mov"].append(np.array([x.cooldown_mov_penalty for x in ag], np.float64))
        rec["time_passed"].append(env.time_passed)
        hit_body = ag.index(lst.fixture.body.userData) if lst.fixture is not None else -1
        rec["listener"].append(np.array([int(lst.hit), hit_body], np.int32))
        if env.done:
            break
    for k, v in rec.items():
        out[k] = np.array(v) if k in ("done", "winner", "time_passed") else np.stack(v)
    meta = dict(name=sc["name"], seed=sc["seed"], n_agents=sc["n_agents"], N=N, steps=len(rec["done"]),
                policy=sc["policy"], note=TDM_NOTE,
                settings=dict(hz=st.hz, time_limit=st.time_limit, cooldown_atk=st.cooldown_atk,
                              cooldown_mov_penalty=st.cooldown_mov_penalty, world_width=env.world_width,
                              world_height=env.world_height))
    out["meta"] = np.array(json.dumps(meta))
    return out


def main():
    gym_stub.install()
    box2d_facade.install()
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "test_scripts"))
    names = sys.argv[1:]
    for sc in SCENARIOS:
        if names and sc["name"] not in names:
            continue
        out = run(sc)
        path = os.path.join(HERE, sc["name"] + ".npz")
        np.savez_compressed(path, **out)
        print(f"{sc['name']}: {os.path.getsize(path)} bytes, collisions={int((out['reward'] < 0).sum())}, "
              f"positive={int((out['reward'] > 0).sum())}, done_steps={int(out['done'].sum())}")
    for sc in TDM_SCENARIOS:
        if names and sc["name"] not in names:
            continue
        out = run_tdm(sc)
        path = os.path.join(HERE, sc["name"] + ".npz")
        np.savez_compressed(path, **out)
        print(f"{sc['name']}: {os.path.getsize(path)} bytes, steps={len(out['done'])}, "
              f"deaths={int((out['alive'][-1] == 0).sum())}, winner={int(out['winner'][-1])}, "
              f"hits={int((np.diff(out['health'], axis=0) < 0).sum())}")


if __name__ == "__main__":
    main()
