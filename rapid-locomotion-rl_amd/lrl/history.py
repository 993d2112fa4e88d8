"""HistoryWrapper (mini_gym/envs/wrappers/history_wrapper.py:6-41) over LeggedRobotEnv.

The 15-step observation history lives in the sim ([N, 15*num_obs] HBM buffer) and is shifted
inside the fused step kernel (LRL_STEP_HISTORY), so ``step`` costs no extra launch.  Attribute
reads fall through to the wrapped env like gym 0.19's ``Wrapper.__getattr__``; attribute WRITES
land on the wrapper (which is why ``Runner.learn(init_at_random_ep_len=True)`` does not reach the
env in the reference either — SURVEY.md Q5).
"""
import torch


class HistoryWrapper:
    def __init__(self, env):
        self.env = env
        self.obs_history_length = self.env.cfg.env.num_observation_history
        self.num_obs_history = self.obs_history_length * self.env.num_obs
        self.obs_history = self.env.obs_history_buf
        self.num_privileged_obs = self.env.num_privileged_obs

    def __getattr__(self, name):
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    def step(self, action):
        obs, rew, done, info = self.env.step(action, _history=True)
        privileged_obs = info["privileged_obs"]
        return {"obs": obs, "privileged_obs": privileged_obs, "obs_history": self.obs_history}, rew, done, info

    def get_observations(self):
        obs = self.env.get_observations()
        privileged_obs = self.env.get_privileged_observations()
        self.env.shift_history()  # history_wrapper.py:29 (Q6: get_observations shifts the history)
        return {"obs": obs, "privileged_obs": privileged_obs, "obs_history": self.obs_history}

    def reset_idx(self, env_ids):
        ret = self.env.reset_idx(env_ids)
        self.obs_history[torch.as_tensor(env_ids, device=self.obs_history.device).long(), :] = 0
        return ret

    def reset(self):
        ret = self.env.reset()
        privileged_obs = self.env.get_privileged_observations()
        self.obs_history[:, :] = 0
        return {"obs": ret, "privileged_obs": privileged_obs, "obs_history": self.obs_history}
