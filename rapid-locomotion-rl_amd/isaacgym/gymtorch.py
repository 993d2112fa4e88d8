"""``isaacgym.gymtorch``: the native sim hands out torch tensors directly (zero-copy DLPack views of its HBM arena,
lrl/env.py), so wrapping and unwrapping are the identity."""


def wrap_tensor(t, *_, **__):
    return t


def unwrap_tensor(t):
    return t
