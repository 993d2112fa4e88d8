"""CPU baseline env (TEST / BENCH INFRASTRUCTURE, not product): the VecEnv surface the Runner drives
(mini_gym/envs/base/legged_robot.py step / get_observations, wrapped by HistoryWrapper) over the oracle's
float + OpenMP build (oracle/build/liblrl_cpu.so, the same source as oracle/lrl_oracle.c).  bench.py's
``cpu_baseline`` leg times a whole PPO iteration through it with the reference's torch PPO math on the CPU
(lrl.ppo, fused=False) — the reference's own Isaac Gym CPU pipeline is proprietary and absent here.
Fork semantics as the GPU bench (no resets inside step; fallen robots stay down)."""
import numpy as np
import torch

from . import oracle


class CpuVecEnv:
    def __init__(self, n, seed=1234, threads=1):
        from lrl import _abi
        from lrl import config as lcfg
        from lrl import params as lparams
        from lrl.robot import load_robot
        cfg = lcfg.make_cfg()
        lcfg.config_mini_cheetah(cfg)
        cfg.terrain.x_offset = 0
        rob = load_robot("mini_cheetah.urdf")
        self.P, self.M = lparams.build_params(cfg, rob), lparams.build_model(rob)
        P, M = self.P, self.M
        self.lib = oracle.cpu_lib()
        self.threads = self.lib.lrlo_set_threads(threads)
        self.flags = _abi.STEP_PHYSICS | _abi.STEP_HISTORY
        self.num_envs = self.num_train_envs = n
        self.num_obs, self.num_privileged_obs = P.num_obs, 18
        self.num_obs_history = P.num_obs * P.num_history
        self.num_actions = 12
        self.max_episode_length = 1001
        st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
        rng = np.random.default_rng(seed)
        st["root"][:, 2] = 0.32
        st["root"][:, :2] = rng.uniform(10, 60, (n, 2))
        st["dof_pos"][:] = np.array(P.default_dof_pos[:], np.float32)
        st["friction"][:] = 1.0
        st["commands"][:, :3] = rng.uniform(-0.6, 0.6, (n, 3)).astype(np.float32)
        self.st = st
        self.counter = 0
        self.episode_length_buf = torch.from_numpy(st["episode_length"])
        self._bins = torch.zeros(n, dtype=torch.long)

    def _obs(self):
        s = self.st
        return {"obs": torch.from_numpy(s["obs"]), "privileged_obs": torch.from_numpy(s["priv"]),
                "obs_history": torch.from_numpy(s["hist"])}

    def get_observations(self):
        return self._obs()

    def reset(self):
        return self._obs()

    def reset_evaluation_envs(self):
        pass

    def step(self, actions):
        self.counter += 1
        oracle.env_step(self.M, self.P, self.st, actions.detach().numpy(), self.flags,
                        common_step_counter=self.counter, library=self.lib)
        s = self.st
        return (self._obs(), torch.from_numpy(s["rew"]), torch.from_numpy(s["reset"].astype(np.int64)),
                {"env_bins": self._bins})


def cpu_compute_returns(storage):
    """GAE + advantage normalisation on the CPU for the baseline's storage (mini_gym_learn/ppo/rollout_storage.py:
    76-90, the reference's loop); bound over RolloutStorage.compute_returns, whose product form is lrl_gae."""
    def compute_returns(last_values, gamma, lam, reduce_stats=None):
        s = storage
        adv = 0
        for step in reversed(range(s.num_transitions_per_env)):
            nv = last_values if step == s.num_transitions_per_env - 1 else s.values[step + 1]
            nt = 1.0 - s.dones[step].float()
            delta = s.rewards[step] + nt * gamma * nv - s.values[step]
            adv = delta + nt * gamma * lam * adv
            s.returns[step] = adv + s.values[step]
        a = s.returns - s.values
        s.advantages.copy_((a - a.mean()) / (a.std() + 1e-8))
    return compute_returns
