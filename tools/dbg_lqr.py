import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from oracle import oracle as O
from cartpoleplusplus_amd.lqr import exact_gains
import test_gpu_lqr as T
B = 128
gpu, orc = T._pair(O, num_envs=B, action_repeats=3, initial_force=55.0, seed=21, autoreset=1)
rng = np.random.default_rng(5)
K = (exact_gains()[None] * rng.uniform(0.0, 1.5, (B, 1, 1, 8))).astype(np.float32)
gpu.enable_lqr(torch.from_numpy(K), per_env=True, done_pos=0.02, done_angle=0.02)
orc.set_lqr(K, per_env=True, state8=True, done_pos=0.02, done_angle=0.02)
gpu.reset(); orc.reset()
a = rng.uniform(-0.3, 0.3, (B, 2, 2)).astype(np.float32)
go, gr, gd = gpu.step(torch.from_numpy(a).cuda()); oo, orw, od = orc.step(a)
g8 = gpu.state8.cpu().numpy(); o8 = orc.state8
d = np.abs(g8 - o8) > 0
print("obs equal", np.array_equal(go.cpu().numpy(), oo))
envs = np.nonzero(d.any(axis=(1,2,3,4)))[0]
print("bad envs", envs[:40], len(envs))
e = envs[0]
np.set_printoptions(precision=4, suppress=True, linewidth=200)
print("gpu", g8[e, :, 0]); print("orc", o8[e, :, 0])
print("sweeps", orc.sweeps()[envs[:10]] if hasattr(orc, 'sweeps') else None)
