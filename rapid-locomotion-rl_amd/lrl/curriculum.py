"""Grid-adaptive command curriculum (host side, numpy) — bit-exact with the reference.

Restates ``Curriculum`` / ``RewardThresholdCurriculum`` (mini_gym/envs/base/curriculum.py:16-124):
a 3-D grid of command bins (lin_vel_x, lin_vel_y, ang_vel_yaw) with sampling weights, sampled with
``np.random.RandomState`` (MT19937) so that ``sample``/``update`` reproduce the reference's draws
bit for bit for the same seed.  This is bookkeeping on a few thousand bins once per resampling
interval; it stays on the host like the reference.
"""
import ctypes as C
import os

import numpy as np


def _native_lib():
    """liblrl.so for the native sample / update (csrc/lrl_curriculum.cpp, bit-exact with the numpy form below), or None
    when the library has not been built (the numpy form then runs; a stale build still raises in _abi.lib())."""
    from . import _abi
    if not os.path.exists(_abi.LIB_PATH):
        return None
    return _abi.lib()


class GridCurriculum:
    """Curriculum (curriculum.py:16-68).  The generator is numpy's RandomState(seed); its MT19937 state lives in
    ``_mt_key`` / ``_mt_pos`` so the native sample (lrl_curriculum_sample) and ``rng`` (a RandomState materialised
    on access, read back before the next native draw) continue one stream."""

    def __init__(self, seed, **key_ranges):
        st = np.random.RandomState(seed).get_state()
        self._mt_key = np.array(st[1], dtype=np.uint32)
        self._mt_pos = np.array([st[2]], dtype=np.int32)
        self._rng_obj = None
        self._native = _native_lib() is not None  # (a flag, not the library: the object stays deep-copyable)
        self.cfg = {k: np.linspace(*r) for k, r in key_ranges.items()}
        self.bin_sizes = {k: a[1] - a[0] for k, a in self.cfg.items()}
        self._raw_grid = np.stack(np.meshgrid(*self.cfg.values(), indexing="ij"))
        self.keys = list(key_ranges)
        self.grid = self._raw_grid.reshape([len(self.keys), -1])
        self._l = self.grid.shape[1]
        self.ls = {k: len(v) for k, v in self.cfg.items()}
        self.weights = np.zeros(self._l)
        self.indices = np.arange(self._l)

    def __len__(self):
        return self._l

    _CACHES = ("_grid_c", "_half_c", "_ptrs", "_axes_c", "_axes_p", "_axes_n")

    def __getstate__(self):
        """copy / deepcopy / pickle: without the cached native pointers (they address this object's arrays)."""
        st = dict(self.__dict__)
        for k in self._CACHES:
            st.pop(k, None)
        return st

    @property
    def rng(self):
        """The curriculum's numpy RandomState (curriculum.py:20), at the current point of the stream."""
        if self._rng_obj is None:
            r = np.random.RandomState()
            r.set_state(("MT19937", self._mt_key, int(self._mt_pos[0])))
            self._rng_obj = r
        return self._rng_obj

    @rng.setter
    def rng(self, r):
        self._rng_obj = r

    def _sync_from_rng(self):
        """Draws made through ``rng`` since it was materialised: take its state back before a native draw."""
        if self._rng_obj is not None:
            st = self._rng_obj.get_state()
            self._mt_key[:] = st[1]
            self._mt_pos[0] = st[2]
            self._rng_obj = None

    def set_to(self, low, high, value=1.0):
        inside = np.logical_and(self.grid >= low[:, None], self.grid <= high[:, None]).all(axis=0)
        self.weights[inside] = value

    def sample_bins(self, batch_size):
        inds = self.rng.choice(self.indices, batch_size, p=self.weights / self.weights.sum())
        return self.grid.T[inds], inds

    def sample_uniform_from_cell(self, centroids):
        half = np.array(list(self.bin_sizes.values())) / 2
        return self.rng.uniform(centroids + half, centroids - half)

    def sample(self, batch_size):
        """One ``uniform`` call over the [batch, 3] cell bounds: RandomState draws one double per element in C
        order, i.e. exactly the per-row calls of curriculum.py:66-68 (np.stack over rows) in sequence.  Three command
        axes and the library present: lrl_curriculum_sample does the choice and the uniform draws natively."""
        if self._native and len(self.keys) == 3 and batch_size > 0:
            from . import _abi
            self._sync_from_rng()
            w = self.weights
            if w.dtype != np.float64 or not w.flags.c_contiguous:
                w = np.ascontiguousarray(w, dtype=np.float64)
            if not hasattr(self, "_grid_c"):  # (persistent arrays: their addresses are taken once)
                self._grid_c = np.ascontiguousarray(self.grid, dtype=np.float64)
                self._half_c = np.ascontiguousarray(np.array(list(self.bin_sizes.values()), np.float64) / 2)
                self._ptrs = tuple(C.c_void_p(a.ctypes.data) for a in (self._mt_key, self._mt_pos, self._grid_c,
                                                                       self._half_c))
            cmds = np.empty((batch_size, 3), np.float64)
            inds = np.empty(batch_size, np.int64)
            k, ps, g, h = self._ptrs
            L = _abi.lib()
            rc = L.lrl_curriculum_sample(k, ps, C.c_void_p(w.ctypes.data), self._l, g, h, batch_size,
                                         C.c_void_p(cmds.ctypes.data), C.c_void_p(inds.ctypes.data))
            if rc != 0:
                raise ValueError(L.lrl_last_error().decode())
            return cmds, inds
        cents, inds = self.sample_bins(batch_size)
        if len(cents) == 0:
            raise ValueError("need at least one array to stack")  # as np.stack([]) in the reference
        return self.sample_uniform_from_cell(cents), inds


class RewardThresholdCurriculum(GridCurriculum):
    """RewardThresholdCurriculum (curriculum.py:92-124)."""

    def __init__(self, seed, **kw):
        super().__init__(seed, **kw)
        n = len(self)
        self.episode_reward_lin = np.zeros(n)
        self.episode_reward_ang = np.zeros(n)
        self.episode_lin_vel_raw = np.zeros(n)
        self.episode_ang_vel_raw = np.zeros(n)
        self.episode_duration = np.zeros(n)

    def get_local_bins(self, bin_inds, range=0.1):
        g = self.grid[:, None, :].repeat(len(bin_inds), axis=1)
        c = self.grid[:, bin_inds, None]
        return np.logical_and(g >= c - range, g <= c + range).all(axis=0)

    def update(self, bin_inds, lin_vel_rewards, ang_vel_rewards, lin_vel_threshold, ang_vel_threshold,
               local_range=0.5):
        """curriculum.py:105-115 with the same result, element for element.  The reference adds 0.2 (clipped to 1)
        to the successful bins, then once per successful entry to every bin of its +-local_range neighbourhood —
        a [3, n_ok, bins] comparison and a Python loop over the entries.  A bin's updates are all the same clipped
        add, so only their COUNT matters: the neighbourhood is a product of per-axis memberships (the same float
        comparisons on the same grid values), the counts are one einsum over the entries, and the clipped add is
        applied count times per bin."""
        self.episode_reward_lin[bin_inds] = lin_vel_rewards
        self.episode_reward_ang[bin_inds] = ang_vel_rewards
        ok = (lin_vel_rewards > lin_vel_threshold) * (ang_vel_rewards > ang_vel_threshold)
        centres = bin_inds[ok]
        if (self._native and len(self.keys) == 3 and self.weights.dtype == np.float64
                and self.weights.flags.c_contiguous):  # lrl_curriculum_update_weights: the same adds, natively
            from . import _abi
            if not hasattr(self, "_axes_c"):
                self._axes_c = np.ascontiguousarray(np.concatenate([self.cfg[k] for k in self.keys]), np.float64)
                self._axes_p = C.c_void_p(self._axes_c.ctypes.data)
                self._axes_n = tuple(self.ls[k] for k in self.keys)
            cen = np.ascontiguousarray(centres, dtype=np.int64)
            nx, ny, nz = self._axes_n
            _abi.check(_abi.lib().lrl_curriculum_update_weights(
                C.c_void_p(self.weights.ctypes.data), self._axes_p, nx, ny, nz, C.c_void_p(cen.ctypes.data), len(cen),
                C.c_double(float(local_range))))
            return
        self.weights[bin_inds[ok]] = np.clip(self.weights[bin_inds[ok]] + 0.2, 0, 1)
        if len(centres) == 0:
            return
        if len(self.keys) != 3:  # (the einsum below is written for the three command axes)
            for adj in self.get_local_bins(centres, range=local_range):
                idx = np.array(adj.nonzero()[0])
                self.weights[idx] = np.clip(self.weights[idx] + 0.2, 0, 1)
            return
        shape = tuple(self.ls[k] for k in self.keys)
        cidx = np.unravel_index(centres, shape)
        member = []
        for d, k in enumerate(self.keys):
            v = self.cfg[k]  # the axis' grid values (self.grid holds exactly these)
            c = v[cidx[d]][:, None]
            member.append(np.logical_and(v[None, :] >= c - local_range, v[None, :] <= c + local_range))
        m01 = (member[0][:, :, None] & member[1][:, None, :]).reshape(len(centres), -1).astype(np.float64)
        counts = (m01.T @ member[2].astype(np.float64)).reshape(-1)  # exact small integers
        idx = np.flatnonzero(counts > 0)
        cnt = counts[idx]
        step = 1
        while len(idx):  # the step-th add reaches the bins counted at least step times; 1.0 is a fixed point
            w = np.clip(self.weights[idx] + 0.2, 0, 1)
            self.weights[idx] = w
            keep = (cnt > step) & (w < 1.0)
            idx, cnt = idx[keep], cnt[keep]
            step += 1

    def _update_literal(self, bin_inds, lin_vel_rewards, ang_vel_rewards, lin_vel_threshold, ang_vel_threshold,
                        local_range=0.5):
        """curriculum.py:105-115 as written (the check for ``update``)."""
        self.episode_reward_lin[bin_inds] = lin_vel_rewards
        self.episode_reward_ang[bin_inds] = ang_vel_rewards
        ok = (lin_vel_rewards > lin_vel_threshold) * (ang_vel_rewards > ang_vel_threshold)
        self.weights[bin_inds[ok]] = np.clip(self.weights[bin_inds[ok]] + 0.2, 0, 1)
        for adj in self.get_local_bins(bin_inds[ok], range=local_range):
            idx = np.array(adj.nonzero()[0])
            self.weights[idx] = np.clip(self.weights[idx] + 0.2, 0, 1)

    def log(self, bin_inds, lin_vel_raw=None, ang_vel_raw=None, episode_duration=None):
        self.episode_lin_vel_raw[bin_inds] = lin_vel_raw.cpu().numpy()
        self.episode_ang_vel_raw[bin_inds] = ang_vel_raw.cpu().numpy()
        self.episode_duration[bin_inds] = episode_duration.cpu().numpy()
