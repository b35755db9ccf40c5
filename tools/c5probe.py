import sys, time, json, torch
sys.path.insert(0, 'gym-macm_amd')
from gym_macm.vec import FlockVec
res = {}
for name, kw in (("default", {}), ("vi0", dict(velocityIterations=0)), ("vi0pi0", dict(velocityIterations=0, positionIterations=0)),
                 ("pi0", dict(positionIterations=0))):
    v = FlockVec(2048, n_agents=[1024], seed=1, device="cuda:0", **kw)
    a = torch.randint(0, 3, (2048, 1024, 3), dtype=torch.uint8, device="cuda:0")
    for _ in range(2): v.step(a)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(4): v.step(a)
    torch.cuda.synchronize(); res[name] = (time.perf_counter() - t) / 4 * 1e3
    del v
print(json.dumps(res))
