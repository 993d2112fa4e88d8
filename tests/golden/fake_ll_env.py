"""A scripted low-level env for the HighLevelControlWrapper parity fixture (tests/golden/make_golden.py and
tests/test_high_level.py): base positions / velocities and low-level dones follow a fixed seeded trajectory;
reset_idx puts the reset envs back at their origin.  Test infrastructure only."""
import numpy as np
import torch


class FakeLowLevelEnv:
    def __init__(self, n=32, T=40, seed=5, device="cpu"):
        rng = np.random.default_rng(seed)
        self.num_envs, self.device, self.dt = n, device, 0.019999999552965164
        f = lambda a: torch.tensor(np.asarray(a, np.float32), device=device)
        self.env_origins = f(rng.uniform(-5, 5, (n, 3)))
        self.base_init_state = f(np.r_[[0.0, 0.0, 0.34, 0, 0, 0, 1], np.zeros(6)])
        # per-step displacement, velocities; a few envs walk straight to the goal (3, 0) so the goal terminal fires
        self.step_disp = f(rng.normal(0, 0.05, (T, n, 3)))
        self.step_disp[:, :4, 0] = 0.25
        self.step_disp[:, :4, 1:] = 0.0
        self.lin = f(rng.normal(0, 0.5, (T, n, 3)))
        self.ang = f(rng.normal(0, 0.5, (T, n, 3)))
        d = rng.random((T, n)) < 0.03
        self.dones_seq = torch.tensor(d, device=device)
        self.root_states = torch.zeros(n, 13, device=device)
        self.root_states[:, :3] = self.env_origins + self.base_init_state[:3]
        self.base_lin_vel = torch.zeros(n, 3, device=device)
        self.base_ang_vel = torch.zeros(n, 3, device=device)
        self.commands = torch.zeros(n, 4, device=device)
        self.rew_buf = torch.zeros(n, device=device)
        self.t = 0
        self.commands_log, self.reset_log = [], []

    def _obs(self):
        return {"obs": torch.zeros(self.num_envs, 42, device=self.device), "privileged_obs": None,
                "obs_history": torch.zeros(self.num_envs, 630, device=self.device)}

    def reset(self):
        return self._obs()

    def step(self, actions):
        t = self.t
        self.commands_log.append(self.commands[:, :3].clone())
        self.root_states[:, :3] += self.step_disp[t]
        self.base_lin_vel[:] = self.lin[t]
        self.base_ang_vel[:] = self.ang[t]
        self.t += 1
        return self._obs(), self.rew_buf, self.dones_seq[t].clone(), {}

    def reset_idx(self, env_ids):
        self.reset_log.append(env_ids.clone())
        self.root_states[env_ids, :3] = self.env_origins[env_ids] + self.base_init_state[:3]
