"""Phase breakdown of the env step kernel under the bench's own workload (bench.py main: 4096 Mini Cheetah envs, the
random-init PPO policy acting, fork semantics), after 2 warm-up iterations; run with LRL_LIB=<the -DLRL_ENV_PROFILE
build> (`make -C rapid-locomotion-rl_amd/csrc liblrl_prof.so`).  argv: [iterations] [self_collisions 0 = on]."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import _abi  # noqa: E402
from lrl import config as lcfg  # noqa: E402
from lrl.env import LeggedRobotEnv  # noqa: E402
from lrl.history import HistoryWrapper  # noqa: E402
from lrl.ppo import runner as R  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = 4096
cfg = lcfg.make_cfg()
lcfg.config_mini_cheetah(cfg)
if "LRL_SOLVER_TYPE" in os.environ:  # 1 = TGS (the presets), 0 = PGS
    cfg.sim.physx.solver_type = int(os.environ["LRL_SOLVER_TYPE"])
if len(sys.argv) > 2:
    cfg.asset.self_collisions = int(sys.argv[2])
cfg.env.num_envs = n
R.RunnerArgs.save_interval = 0
R.RunnerArgs.log_freq = 10 ** 9
env = HistoryWrapper(LeggedRobotEnv("cuda:0", cfg=cfg, seed=1234))
g = torch.Generator(device="cuda:0").manual_seed(1)
cmd = torch.rand(n, 3, device="cuda:0", generator=g)
env.env.commands[:, 0] = cmd[:, 0] * 1.2 - 0.6
env.env.commands[:, 1] = cmd[:, 1] * 1.2 - 0.6
env.env.commands[:, 2] = cmd[:, 2] * 2.0 - 1.0
runner = R.Runner(env, device="cuda:0", seed=1234)
runner.learn(2, init_at_random_ep_len=True)
torch.cuda.synchronize()
L = _abi.lib()
buf = (C.c_ulonglong * 24)()
L.lrl_debug_env_profile(buf, 1)
runner.learn(iters)
torch.cuda.synchronize()
assert L.lrl_debug_env_profile(buf, 0) >= 16, "library built without LRL_ENV_PROFILE"
K = 24 * iters
waves = (n + 3) // 4  # the plane kernel: 4 envs per wave (16 lanes per env); profiles r6t and earlier divided by n / 16
names = ["kin+dyn+detect", "schur+free acc", "delassus+warm", "PGS", "integrate", "start+state load", "post-physics",
         "tiles+history", "PD torques"]
tot = sum(buf[:9])
for i, nm in enumerate(names):
    print(f"{nm:16s} {buf[i] / waves / K:10.0f} cycles/wave/step  {100 * buf[i] / tot:5.1f}%")
for i, nm in zip(range(10, 14), ["  contact forces", "  loads/teleport/DR", "  rewards+sums", "  obs/priv rows"]):
    print(f"{nm:16s} {buf[i] / waves / K:10.0f} cycles/wave/step  (part of post-physics)")
if buf[14]:
    print(f"  self detect     {buf[14] / waves / K:10.0f} cycles/wave/step; LDS pass entered "
          f"{buf[15] / waves / K:.3f} times per wave and step")
base = env.env.root_states
print(f"total {tot / waves / K:.0f} cycles/wave/step (wave lifetime {buf[9] / waves / K:.0f}); base z mean "
      f"{base[:, 2].mean().item():.3f}, upright {(env.env.projected_gravity[:, 2] < -0.5).float().mean().item():.3f}")
