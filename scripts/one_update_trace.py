import sys, os
sys.path.insert(0, "rapid-locomotion-rl_amd")
import torch
from lrl.ppo.actor_critic import ActorCritic
from lrl.ppo.ppo import PPO
N, T = 4096, 24
ac = ActorCritic(42, 18, 630, 12)
alg = PPO(ac.cuda(), device="cuda:0", fused=True)
alg.init_storage(N, T, [42], [18], [630], [12])
st = alg.storage
with torch.no_grad():
    for name in ("observations", "privileged_observations", "observation_histories", "actions", "mu", "values", "returns", "advantages"):
        getattr(st, name).copy_(torch.randn(getattr(st, name).shape, device="cuda:0"))
    st.sigma.fill_(1.0); st.actions_log_prob.fill_(-11.0)
st.step = T
print("---- update", file=sys.stderr)
alg.update()
torch.cuda.synchronize()
