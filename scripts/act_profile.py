"""Phase breakdown of the one-launch act (act_fused_kernel; build with `make -C rapid-locomotion-rl_amd/csrc
liblrl_prof.so PROF_DEFS=-DLRL_ACT_PROFILE`, run with LRL_LIB=<that build> LRL_ACT_FUSED=1): shader-clock cycles per
workgroup and act for each phase, 4096 rows, the preset network.  usage: python scripts/act_profile.py [acts]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rapid-locomotion-rl_amd"))
import torch  # noqa: E402

from lrl import _abi  # noqa: E402
from lrl.ppo.actor_critic import ActorCritic  # noqa: E402
from lrl.ppo.rollout_storage import RolloutStorage  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
n = 4096
ac = ActorCritic(42, 18, 630, 12).cuda()
st = RolloutStorage(n, 24, [42], [18], [630], [12], "cuda:0")
g = torch.Generator(device="cuda:0").manual_seed(0)
obs = torch.randn(n, 42, device="cuda:0", generator=g)
priv = torch.randn(n, 18, device="cuda:0", generator=g)
hist = torch.randn(n, 630, device="cuda:0", generator=g)
L = _abi.lib()
buf = (C.c_ulonglong * 12)()
for i in range(10):
    ac.act_fused(obs, priv, hist, seed=1, counter=i + 1, store=st.store_desc(), store_row=i % 24)
torch.cuda.synchronize()
assert L.lrl_debug_act_profile(buf, 1) == 12, "library built without LRL_ACT_PROFILE"
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for i in range(K):
    ac.act_fused(obs, priv, hist, seed=1, counter=i + 1, store=st.store_desc(), store_row=i % 24)
ev1.record()
torch.cuda.synchronize()
L.lrl_debug_act_profile(buf, 0)
wgs = (n + 15) // 16
names = ["stage", "enc1", "enc2", "enc3", "ac1", "ac2", "ac3", "heads", "sample", "storage"]
tot = sum(buf[i] for i in range(10))
print(f"act {ev0.elapsed_time(ev1) / K * 1e3:.1f} us per launch (events, {K} launches)")
for i, nm in enumerate(names):
    print(f"{nm:8s} {buf[i] / (wgs * K):10.0f} cycles/WG  {100 * buf[i] / max(tot, 1):5.1f} %")
print(f"{'total':8s} {tot / (wgs * K):10.0f} cycles/WG")
