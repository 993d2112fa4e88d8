"""``isaacgym.torch_utils`` helpers mini_gym calls (legged_robot.py:8: quat_rotate_inverse, quat_apply, to_torch,
torch_rand_float, get_axis_params; math_utils.py:7: quat_apply / normalize).  Quaternions are (x, y, z, w), as in
Isaac Gym; the formulas are legged_gym's (parity unpinned: the module is not vendored)."""
import numpy as np
import torch


def quat_mul(a, b):
    shape = a.shape
    a, b = a.reshape(-1, 4), b.reshape(-1, 4)
    x1, y1, z1, w1 = a.unbind(-1)
    x2, y2, z2, w2 = b.unbind(-1)
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


def _rotate(q, v, sign):
    q_w, q_vec = q[:, -1], q[:, :3]
    a = v * (2.0 * q_w ** 2 - 1.0).unsqueeze(-1)
    b = torch.cross(q_vec, v, dim=-1) * q_w.unsqueeze(-1) * 2.0
    c = q_vec * (q_vec * v).sum(-1, keepdim=True) * 2.0
    return a + b + c if sign > 0 else a - b + c


def quat_rotate(q, v):
    return _rotate(q, v, 1)


def quat_rotate_inverse(q, v):
    return _rotate(q, v, -1)


def quat_apply(a, b):
    shape = b.shape
    a, b = a.reshape(-1, 4), b.reshape(-1, 3)
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
    assert axis_idx < n_dims, "the axis dim should be within the vector dimensions"
    params = np.zeros((n_dims,))
    params[axis_idx] = value
    params[0] = x_value
    return list(params.astype(dtype))


def wrap_to_pi(angles):
    angles = angles % (2 * np.pi)
    return angles - 2 * np.pi * (angles > np.pi)


def copysign(a, b):
    return torch.abs(torch.as_tensor(a, device=b.device, dtype=b.dtype).repeat(b.shape[0])) * torch.sign(b)
