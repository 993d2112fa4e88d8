"""scripts/train.py — the reference's training flow (scripts/train.py:1-54: isaacgym / ml_logger imports, logger.configure
/ log_text / log_params, VelocityTrackingEasyEnv, HistoryWrapper, Runner(env, device), runner.learn) — runs on the GPU
through the package's stand-ins and leaves the run directory the reference's tools read back (play.py: parameters.pkl,
checkpoints/ac_weights_last.pt; the deployment's TorchScript exports)."""
import copy
import importlib.util
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))


@pytest.mark.gpu
def test_reference_train_flow_writes_a_run(tmp_path):
    from ml_logger import logger
    from mini_gym.envs.base.legged_robot_config import Cfg
    from mini_gym_learn.ppo import RunnerArgs
    from mini_gym_learn.ppo.actor_critic import ActorCritic
    saved = copy.deepcopy(Cfg)
    saved_args = dict(save_interval=RunnerArgs.save_interval, log_freq=RunnerArgs.log_freq)
    RunnerArgs.save_interval, RunnerArgs.log_freq = 400, 1  # the reference's defaults (other tests zero them)
    spec = importlib.util.spec_from_file_location("lrl_scripts_train", os.path.join(ROOT, "scripts", "train.py"))
    script = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(script)
    try:
        logger.configure(logger.utcnow("rapid-locomotion/%Y-%m-%d/train/%H%M%S.%f"), root=str(tmp_path))
        logger.log_text("charts: []\n", filename=".charts.yml", dedent=True)
        runner = script.train_mc(headless=True, iterations=2, robot="go1")
        run = logger.run_dir
        params = logger.load_pkl("parameters.pkl")
        assert params[0]["RunnerArgs"]["num_steps_per_env"] == RunnerArgs.num_steps_per_env
        assert params[0]["Cfg"]["env"]["num_envs"] == Cfg.env.num_envs
        for f in ("ac_weights_000000.pt", "ac_weights_000001.pt", "ac_weights_last.pt", "adaptation_module_latest.jit",
                  "body_latest.jit"):
            assert os.path.exists(os.path.join(run, "checkpoints", f)), f
        # play.py's load_env: ActorCritic from the Cfg sizes, the state dict through logger.load_torch
        ac = ActorCritic(num_obs=Cfg.env.num_observations, num_privileged_obs=Cfg.env.num_privileged_obs,
                         num_obs_history=Cfg.env.num_observations * Cfg.env.num_observation_history,
                         num_actions=Cfg.env.num_actions)
        ac.load_state_dict(state_dict=logger.load_torch("checkpoints/ac_weights_last.pt"))
        got = {k: v.cpu() for k, v in ac.state_dict().items()}
        want = {k: v.cpu() for k, v in runner.alg.actor_critic.state_dict().items()}
        assert list(got) == list(want) and all(torch.equal(got[k], want[k]) for k in want)
        runner.env.env.close()
        assert len(logger.load_pkl("metrics.pkl")) == 2  # log_freq 1: one summary per iteration
    finally:
        RunnerArgs.save_interval, RunnerArgs.log_freq = saved_args["save_interval"], saved_args["log_freq"]
        logger.configure(None)
        Cfg.__dict__.clear()
        Cfg.__dict__.update(saved.__dict__)
