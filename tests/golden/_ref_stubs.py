"""Stub modules that let the reference's pure-Python code import in THIS container.

Used only by ``make_golden.py`` (fixture generation, never shipped to / run on the GPU box).
Third-party modules the reference imports but that are absent here:

* ``params_proto`` (PrefixProto config classes) -> plain base class,
* ``ml_logger`` -> ``logger = None``,
* ``gym`` 0.19 (``gym.Env`` / ``gym.Wrapper``) -> minimal classes (``Wrapper`` forwards
  ``__getattr__`` only, as gym 0.19 does),
* ``isaacgym`` (NVIDIA Isaac Gym Preview 3, proprietary, un-vendored) -> empty modules plus a
  restatement of the ``isaacgym.torch_utils`` helpers the reference uses
  (legged_robot.py:8, math_utils.py:7).  These follow the published legged_gym/Isaac Gym
  formulas; no reference test pins them (parity unpinned at that boundary).
"""
import sys
import types

import numpy as np
import torch


def _mod(name, **kw):
    m = types.ModuleType(name)
    m.__dict__.update(kw)
    sys.modules[name] = m
    return m


class PrefixProto:
    def __init_subclass__(cls, **kw):
        pass


class _Env:
    pass


class _Wrapper:
    def __init__(self, env):
        self.env = env

    def __getattr__(self, k):
        return getattr(self.env, k)


# ---- isaacgym.torch_utils restatement (Isaac Gym Preview 3, quaternions are xyzw) ----
def quat_rotate_inverse(q, v):
    shape = q.shape
    q_w = q[:, -1]
    q_vec = q[:, :3]
    a = v * (2.0 * q_w ** 2 - 1.0).unsqueeze(-1)
    b = torch.cross(q_vec, v, dim=-1) * q_w.unsqueeze(-1) * 2.0
    c = q_vec * torch.bmm(q_vec.view(shape[0], 1, 3), v.view(shape[0], 3, 1)).squeeze(-1) * 2.0
    return a - b + c


def quat_rotate(q, v):
    shape = q.shape
    q_w = q[:, -1]
    q_vec = q[:, :3]
    a = v * (2.0 * q_w ** 2 - 1.0).unsqueeze(-1)
    b = torch.cross(q_vec, v, dim=-1) * q_w.unsqueeze(-1) * 2.0
    c = q_vec * torch.bmm(q_vec.view(shape[0], 1, 3), v.view(shape[0], 3, 1)).squeeze(-1) * 2.0
    return a + b + c


def quat_mul(a, b):
    shape = a.shape
    a = a.reshape(-1, 4)
    b = b.reshape(-1, 4)
    x1, y1, z1, w1 = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
    x2, y2, z2, w2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    ww = (z1 + x1) * (x2 + y2)
    yy = (w1 - y1) * (w2 + z2)
    zz = (w1 + y1) * (w2 - z2)
    xx = ww + yy + zz
    qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
    w = qq - ww + (z1 - y1) * (y2 - z2)
    x = qq - xx + (x1 + w1) * (x2 + w2)
    y = qq - yy + (w1 - x1) * (y2 + z2)
    z = qq - zz + (z1 + y1) * (w2 - x2)
    return torch.stack([x, y, z, w], dim=-1).view(shape)


def quat_conjugate(a):
    shape = a.shape
    a = a.reshape(-1, 4)
    return torch.cat((-a[:, :3], a[:, -1:]), dim=-1).view(shape)


def quat_apply(a, b):
    shape = b.shape
    a = a.reshape(-1, 4)
    b = b.reshape(-1, 3)
    xyz = a[:, :3]
    t = xyz.cross(b, dim=-1) * 2
    return (b + a[:, 3:] * t + xyz.cross(t, dim=-1)).view(shape)


def normalize(x, eps: float = 1e-9):
    return x / x.norm(p=2, dim=-1).clamp(min=eps, max=None).unsqueeze(-1)


def torch_rand_float(lower, upper, shape, device):
    return (upper - lower) * torch.rand(*shape, device=device) + lower


def to_torch(x, dtype=torch.float, device="cuda:0", requires_grad=False):
    return torch.tensor(x, dtype=dtype, device=device, requires_grad=requires_grad)


def get_axis_params(value, axis_idx, x_value=0.0, dtype=np.float64, n_dims=3):
    zs = np.zeros((n_dims,))
    assert axis_idx < n_dims, "the axis dim should be within the vector dimensions"
    zs[axis_idx] = 1.0
    params = np.where(zs == 1.0, value, zs)
    params[0] = x_value
    return list(params.astype(dtype))


def install():
    _mod("params_proto")
    _mod("params_proto.neo_proto", PrefixProto=PrefixProto, ParamsProto=PrefixProto, Meta=object)
    _mod("ml_logger", logger=None)
    _mod("gym", Env=_Env, Wrapper=_Wrapper)
    sys.modules["gym"].spaces = _mod("gym.spaces")
    ig = _mod("isaacgym")
    for sub in ["gymapi", "gymtorch", "gymutil", "terrain_utils"]:
        setattr(ig, sub, _mod("isaacgym." + sub))
    names = ["quat_rotate_inverse", "quat_rotate", "quat_mul", "quat_conjugate", "quat_apply",
             "normalize", "torch_rand_float", "to_torch", "get_axis_params"]
    tu = _mod("isaacgym.torch_utils", __all__=names + ["np", "torch"], np=np, torch=torch)
    for n in names:
        setattr(tu, n, globals()[n])
    ig.torch_utils = tu
    np.int = int  # Q12: legged_robot.py:1065 uses np.int (removed in numpy>=1.24)
