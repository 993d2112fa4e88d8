"""mini_gym/utils/math_utils.py helpers (legged_gym formulas; the env kernel restates quat_apply_yaw for the height
scan, lrl_env.hip::height_sample)."""
import numpy as np
import torch
from isaacgym.torch_utils import normalize, quat_apply


def quat_apply_yaw(quat, vec):
    quat_yaw = quat.clone().view(-1, 4)
    quat_yaw[:, :2] = 0.0
    return quat_apply(normalize(quat_yaw), vec)


def wrap_to_pi(angles):
    angles %= 2 * np.pi
    angles -= 2 * np.pi * (angles > np.pi)
    return angles


def torch_rand_sqrt_float(lower, upper, shape, device):
    r = 2 * torch.rand(*shape, device=device) - 1
    r = torch.where(r < 0.0, -torch.sqrt(-r), torch.sqrt(r))
    return (upper - lower) * ((r + 1.0) / 2.0) + lower


def get_scale_shift(rng):
    return 2.0 / (rng[1] - rng[0]), (rng[1] + rng[0]) / 2.0
