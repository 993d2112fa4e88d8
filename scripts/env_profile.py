"""Phase breakdown of the env step kernel (build: -DLRL_ENV_PROFILE, see csrc/lrl_env.hip; run with
LRL_LIB=<that build>).  4096 Mini Cheetah envs, random actions."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import _abi  # noqa: E402
from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cfg = lcfg.make_cfg()
lcfg.config_mini_cheetah(cfg)
env = LeggedRobotEnv("cuda:0", cfg=cfg, num_envs=n)
env.reset()
L = _abi.lib()
buf = (C.c_ulonglong * 14)()
g = torch.Generator(device="cuda:0").manual_seed(0)
for _ in range(50):
    env.step(0.5 * torch.randn(n, 12, device="cuda:0", generator=g), _history=True)
torch.cuda.synchronize()
L.lrl_debug_env_profile(buf, 1)
K = 100
for _ in range(K):
    env.step(0.5 * torch.randn(n, 12, device="cuda:0", generator=g), _history=True)
torch.cuda.synchronize()
assert L.lrl_debug_env_profile(buf, 0) == 14, "library built without LRL_ENV_PROFILE"
waves = (n + 15) // 16  # quad layout: 16 envs per wave
names = ["kin+dyn+detect", "schur+free acc", "delassus+warm", "PGS", "integrate", "start+state load", "post-physics",
         "tiles+history", "PD torques"]
tot = sum(buf[:9])
for i, nm in enumerate(names[:9]):
    print(f"{nm:16s} {buf[i] / waves / K:10.0f} cycles/wave/step  {100 * buf[i] / tot:5.1f}%")
for i, nm in zip(range(10, 14), ["  contact forces", "  loads/teleport/DR", "  rewards+sums", "  obs/priv rows"]):
    print(f"{nm:16s} {buf[i] / waves / K:10.0f} cycles/wave/step  (part of post-physics)")
print(f"total {tot / waves / K:.0f} cycles/wave/step (wave lifetime {buf[9] / waves / K:.0f}); "
      f"resets/step {env._reset_u8.float().mean().item():.3f}")
