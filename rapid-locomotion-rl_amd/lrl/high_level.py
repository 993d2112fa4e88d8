"""HighLevelControlWrapper — the reference's second client of the env API (scripts/high_level_play.py:30-363).

A high-level policy outputs body-velocity commands (3 actions) every policy step; a frozen low-level locomotion
policy turns the env's observations into joint targets; the wrapper keeps its own observation (base position
relative to the start, base velocities, last command, goal), rewards (distance to the goal, action rate,
lateral / backward velocity; terminal rewards for reaching the goal, low-level falls and time-outs), episode
bookkeeping and resets.  All of it is host-side torch on the env's device, as in the reference; the env step and
the low-level policy run on the native path (``LeggedRobotEnv.step`` = one fused HIP launch, the low-level
policy through ``ActorCritic.act_student_fused`` = the adaptation module + actor GEMM chain).

The reference's constructor loads the newest ml_logger run (``_load_env``, :251-334); here the low-level env and
policy are passed in, or built by ``from_actor_critic`` with the evaluation overrides of ``_load_env`` (domain
randomisation off, 3 x 5 terrain tiles, no border).
"""
import torch


class reward_scales:  # high_level_play.py:16-28
    # terminal rewards
    terminal_distance_covered = 0.00
    terminal_distance_gs = 5.0
    terminal_ll_reset = -2.0
    terminal_time_out = -1.0
    # step rewards
    distance = -0.1
    action_rate = -0.01
    lateral_vel = -0.05
    backward_vel = -0.005


class HighLevelControlWrapper:
    def __init__(self, ll_env, low_level_policy, num_envs=None, device=None, goal=(3.0, 0.0)):
        """ll_env: a HistoryWrapper over LeggedRobotEnv; low_level_policy: obs dict -> joint actions."""
        self.ll_env = ll_env
        self.low_level_policy = low_level_policy
        self.device = device or ll_env.device
        self.num_obs = 14
        self.num_actions = 3
        self.max_episode_length_s = 10
        self.num_privileged_obs = 18
        self.num_obs_history = 16
        self.num_envs = num_envs or ll_env.num_envs
        self.num_train_envs = max(1, int(self.num_envs * 0.95))
        self.dt = ll_env.dt
        self.max_episode_length = int(self.max_episode_length_s / ll_env.dt)
        self.ll_env.commands[:, :3] = 0.0
        self.ll_obs = self.ll_env.reset()
        self.ll_rew = self.ll_env.rew_buf
        n, d = self.num_envs, self.device
        z = lambda *s, dtype=torch.float: torch.zeros(*s, device=d, dtype=dtype)
        self.obs_buf = z(n, self.num_obs)
        self.rew_buf = z(n)
        self.discount_rew_buf = z(n) + 1.0
        self.gs_buf = z(n, dtype=torch.bool)
        self.reset_buf = z(n, dtype=torch.bool)
        self.time_buf = z(n, dtype=torch.bool)
        self.episode_length_buf = z(n, dtype=torch.int)
        self.actions = z(n, self.num_actions)
        self.last_actions = z(n, self.num_actions)
        self.last_pos = self._base_pos()
        self.dist_travelled = z(n)
        self.lateral_vel = z(n)
        self.backward_vel = z(n)
        self.privileged_obs_buf = z(n, self.num_privileged_obs)
        self.obs_history = z(n, self.num_obs_history)
        self.goal_position = z(n, 2)
        self.goal_position[:, 0] = goal[0]
        self.goal_position[:, 1] = goal[1]
        self.extras = {}
        attrs = {k: v for k, v in vars(reward_scales).items() if not k.startswith("__")}
        self.reward_scales = {k: v for k, v in attrs.items() if not k.startswith("terminal")}
        self.terminal_reward_scales = {k: v for k, v in attrs.items() if k.startswith("terminal")}
        self._prepare_reward_function()

    @classmethod
    def from_actor_critic(cls, actor_critic, num_envs=1, device="cuda:0", robot="go1", seed=0):
        """The environment of _load_env (high_level_play.py:251-334): config_go1 with every domain randomisation
        off, 3 x 5 terrain tiles without border; the low-level policy is ``actor_critic``'s student path."""
        from . import config as lcfg
        from .env import LeggedRobotEnv
        from .history import HistoryWrapper
        cfg = lcfg.make_cfg()
        (lcfg.config_go1 if robot == "go1" else lcfg.config_mini_cheetah)(cfg)
        dr = cfg.domain_rand
        for k in ("push_robots", "randomize_friction", "randomize_restitution", "randomize_motor_strength",
                  "randomize_base_mass", "randomize_Kd_factor", "randomize_Kp_factor", "randomize_com_displacement"):
            setattr(dr, k, False)
        cfg.env.num_envs = num_envs
        cfg.terrain.num_rows, cfg.terrain.num_cols, cfg.terrain.border_size = 3, 5, 0
        cfg.terrain.max_init_terrain_level = min(cfg.terrain.max_init_terrain_level, cfg.terrain.num_rows - 1)
        env = HistoryWrapper(LeggedRobotEnv(device, cfg=cfg, seed=seed))
        actor_critic = actor_critic.to(env.device)

        def policy(ob):  # ActorCritic.act_inference (actor_critic.py:96-99) on the native student path
            return actor_critic.act_student_fused(ob["obs"].contiguous(), ob["obs_history"])[0]

        return cls(env, policy, num_envs=num_envs, device=env.device)

    def _base_pos(self):
        e = self.ll_env
        return e.root_states[:, :3] - e.env_origins[:, :3] - e.base_init_state[:3]

    def _prepare_reward_function(self):
        """high_level_play.py:88-129: zero scales dropped, step rewards x dt, terminal rewards as they are."""
        for key in list(self.reward_scales):
            if self.reward_scales[key] == 0:
                self.reward_scales.pop(key)
            else:
                self.reward_scales[key] *= self.dt
        for key in list(self.terminal_reward_scales):
            if self.terminal_reward_scales[key] == 0:
                self.terminal_reward_scales.pop(key)
        self.reward_names = list(self.reward_scales)
        self.reward_functions = [getattr(self, "_reward_" + k) for k in self.reward_names]
        self.terminal_reward_names = list(self.terminal_reward_scales)
        self.terminal_reward_functions = [getattr(self, "_reward_" + k) for k in self.terminal_reward_names]
        names = [*self.reward_scales, *self.terminal_reward_scales]
        n, d = self.num_envs, self.device
        self.episode_sums = {k: torch.zeros(n, device=d) for k in names}
        self.episode_sums["total"] = torch.zeros(n, device=d)
        self.episode_sums_eval = {k: -torch.ones(n, device=d) for k in names}
        self.episode_sums_eval["total"] = torch.zeros(n, device=d)

    def step(self, actions):
        """high_level_play.py:131-150: the command is clipped to [-2, 2] and its xy part zeroed below 0.2; the
        low-level policy acts on the previous low-level observation, then the env steps with the new command."""
        self.actions = torch.clamp(actions, -2, 2)
        self.actions[:, :2] *= (torch.norm(self.actions[:, :2], dim=1) > 0.2).unsqueeze(1)
        with torch.no_grad():
            ll_actions = self.low_level_policy(self.ll_obs)
        self.ll_env.commands[:, :3] = self.actions
        self.ll_obs, self.ll_rew, self.ll_dones, self.ll_info = self.ll_env.step(ll_actions)
        self.episode_length_buf += 1
        self.post_physics_step()
        env_ids = self.check_termination()
        self.compute_reward()
        self.reset_idx(env_ids)
        self.compute_observations()
        self.last_actions[:] = self.actions[:]
        return self.get_observations(), self.rew_buf, self.reset_buf, self.extras

    def post_physics_step(self):
        self.lateral_vel[:] = 0.0
        self.backward_vel[:] = 0.0
        self.base_pos = self._base_pos()
        self.dist_travelled[:] += torch.abs(torch.linalg.norm(self.base_pos - self.last_pos, dim=-1))
        self.lateral_vel[:] = self.ll_env.base_lin_vel[:, 1]
        self.backward_vel[:] = torch.clamp_max(self.ll_env.base_lin_vel[:, 0], 0)

    def compute_observations(self):
        self.base_pos = self._base_pos()
        self.base_lin_vel = self.ll_env.base_lin_vel
        self.base_ang_vel = self.ll_env.base_ang_vel
        self.obs_buf = torch.cat([self.base_pos, self.base_lin_vel, self.base_ang_vel, self.actions,
                                  self.goal_position], dim=-1)
        self.last_pos[:] = self.base_pos[:]

    def compute_reward(self):
        self.rew_buf[:] = 0.0
        for name, fn in zip(self.reward_names, self.reward_functions):
            rew = fn() * self.reward_scales[name]
            self.rew_buf += rew
            self.episode_sums[name] += rew
        if len(self.reset_buf.nonzero(as_tuple=False)) > 0:  # terminal rewards in steps where some env ends
            for name, fn in zip(self.terminal_reward_names, self.terminal_reward_functions):
                rew = fn() * self.terminal_reward_scales[name]
                self.rew_buf += rew
                self.episode_sums[name] += rew
        self.episode_sums["total"] += self.rew_buf

    def check_termination(self):
        self.gs_buf = torch.linalg.norm(self.base_pos[:, :2] - self.goal_position, dim=-1) < 0.1
        self.time_buf = self.episode_length_buf > self.max_episode_length
        self.reset_buf |= self.ll_dones
        self.reset_buf |= self.gs_buf
        self.reset_buf |= self.time_buf
        return self.reset_buf.nonzero(as_tuple=False).flatten()

    def reset_idx(self, env_ids):
        if len(env_ids) == 0:
            return self.obs_buf
        tr = env_ids[env_ids < self.num_train_envs]
        if len(tr) > 0:
            self.extras["train/episode"] = {}
            for key in self.episode_sums:
                self.extras["train/episode"]["rew_" + key] = torch.mean(self.episode_sums[key][tr])
                self.episode_sums[key][tr] = 0
        ev = env_ids[env_ids >= self.num_train_envs]
        if len(ev) > 0:
            self.extras["eval/episode"] = {}
            for key in self.episode_sums_eval:
                unset = ev[self.episode_sums_eval[key][ev] == -1]
                self.episode_sums_eval[key][unset] = self.episode_sums[key][unset]
                self.extras["eval/episode"]["rew_" + key] = torch.mean(self.episode_sums[key][ev])
                self.episode_sums[key][ev] = 0
        self.ll_env.reset_idx(env_ids)
        self.rew_buf[env_ids] = 0.0
        self.episode_length_buf[env_ids] = 0
        self.lateral_vel[env_ids] = 0.0
        self.backward_vel[env_ids] = 0.0
        self.dist_travelled[env_ids] = 0.0
        e = self.ll_env
        self.last_pos[env_ids] = e.root_states[env_ids, :3] - e.env_origins[env_ids, :3] - e.base_init_state[:3]
        self.compute_observations()
        self.reset_buf[env_ids] = False
        return self.get_observations()

    def reset(self):
        self.reset_idx(torch.arange(0, self.num_envs, 1, dtype=torch.long, device=self.device))
        return self.get_observations()

    def reset_evaluation_envs(self):
        ids = torch.arange(self.num_train_envs, self.num_envs, 1, dtype=torch.long, device=self.device)
        self.extras.setdefault("eval/episode", {})
        for key in self.episode_sums_eval:
            unset = ids[self.episode_sums_eval[key][ids] == -1]
            self.episode_sums_eval[key][unset] = self.episode_sums[key][unset]
            s = self.episode_sums_eval[key]
            self.extras["eval/episode"]["rew_" + key] = torch.mean(s[s != -1])
        self.reset_idx(ids)
        for key in self.episode_sums_eval:
            self.episode_sums_eval[key] = -torch.ones(self.num_envs, device=self.device)
        return self.get_observations()

    def get_observations(self):
        return {"obs": self.obs_buf, "privileged_obs": self.privileged_obs_buf, "obs_history": self.obs_history}

    # ---- rewards (high_level_play.py:339-363) ----
    def _reward_distance(self):
        return torch.linalg.norm(self.last_pos[:, :2] - self.goal_position, dim=-1)

    def _reward_lateral_vel(self):
        return torch.square(self.lateral_vel)

    def _reward_backward_vel(self):
        return torch.square(self.backward_vel)

    def _reward_action_rate(self):
        return torch.sum(torch.square(self.last_actions - self.actions), dim=1)

    def _reward_terminal_ll_reset(self):
        return self.ll_dones * 1.0

    def _reward_terminal_distance_gs(self):
        return self.gs_buf * 1.0

    def _reward_terminal_distance_covered(self):
        return self.dist_travelled

    def _reward_terminal_time_out(self):
        return self.time_buf * 1.0
