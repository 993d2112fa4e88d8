"""Phase breakdown of the env step kernel (build: -DLRL_ENV_PROFILE, see csrc/lrl_env.hip; run with
LRL_LIB=<that build>, e.g. `make -C rapid-locomotion-rl_amd/csrc liblrl_prof.so`).  4096 envs, random actions;
argv: [n] [mc | go1 | go1_rough]."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import _abi  # noqa: E402
from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
which = sys.argv[2] if len(sys.argv) > 2 else "mc"
cfg = lcfg.make_cfg()
(lcfg.config_mini_cheetah if which == "mc" else lcfg.config_go1)(cfg)
if os.environ.get("LRL_SELF") == "0":
    cfg.asset.self_collisions = 1  # off
if which == "go1_rough":
    cfg.terrain.mesh_type = "trimesh"
    cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
    cfg.terrain.curriculum = True
env = LeggedRobotEnv("cuda:0", cfg=cfg, num_envs=n)
env.reset()
L = _abi.lib()
buf = (C.c_ulonglong * 24)()
g = torch.Generator(device="cuda:0").manual_seed(0)
for _ in range(50):
    env.step(float(os.environ.get("LRL_ASTD", "0.5")) * torch.randn(n, 12, device="cuda:0", generator=g), _history=True)
torch.cuda.synchronize()
L.lrl_debug_env_profile(buf, 1)
K = 100
for _ in range(K):
    env.step(float(os.environ.get("LRL_ASTD", "0.5")) * torch.randn(n, 12, device="cuda:0", generator=g), _history=True)
torch.cuda.synchronize()
assert L.lrl_debug_env_profile(buf, 0) >= 16, "library built without LRL_ENV_PROFILE"
epw = 16 if which == "go1_rough" else 4  # envs per wave: the mesh kernel 16, the plane kernel 4 (16 lanes per env)
waves = (n + epw - 1) // epw
names = ["kin+dyn+detect", "schur+free acc", "delassus+warm", "PGS", "integrate", "start+state load", "post-physics",
         "tiles+history", "PD torques"]
tot = sum(buf[:9])
for i, nm in enumerate(names[:9]):
    print(f"{nm:16s} {buf[i] / waves / K:10.0f} cycles/wave/step  {100 * buf[i] / tot:5.1f}%")
for i, nm in zip(range(10, 14), ["  contact forces", "  loads/teleport/DR", "  rewards+sums", "  obs/priv rows"]):
    print(f"{nm:16s} {buf[i] / waves / K:10.0f} cycles/wave/step  (part of post-physics)")
if which != "go1_rough" and buf[14]:
    print(f"  self detect     {buf[14] / waves / K:10.0f} cycles/wave/step  (part of kin+dyn+detect); LDS pass entered "
          f"{buf[15] / waves / K:.3f} times per wave and step")
if which == "go1_rough" and buf[15]:
    print(f"  terrain queries {buf[14] / waves / K:10.0f} cycles/wave/step  ({buf[15] / waves / K:.1f} per lane, "
          f"{buf[14] / buf[15]:.0f} cycles each; part of kin+dyn+detect)")
if which == "go1_rough" and buf[20]:
    print(f"  query rounds    {buf[20] / waves / K:10.2f} per wave and step; per round: gathers {buf[16] / buf[20]:.0f} "
          f"cycles, walk {buf[17] / buf[20]:.0f} cycles over {buf[18] / buf[20]:.1f} iterations "
          f"({buf[17] / max(buf[18], 1):.0f} cycles each); lane 0 marked {buf[19] / buf[20]:.1f} triangles per query, "
          f"{buf[21] / buf[20]:.2f} of its queries ended at the max-height test")
    print(f"  scan+publish    {buf[22] / waves / K:10.0f} cycles/wave/step; activation {buf[23] / waves / K:.0f}; "
          f"rounds outside the query {(buf[14] - buf[22] - buf[23] - buf[16] - buf[17]) / waves / K:.0f}")
print(f"total {tot / waves / K:.0f} cycles/wave/step (wave lifetime {buf[9] / waves / K:.0f}); "
      f"resets/step {env._reset_u8.float().mean().item():.3f}")
