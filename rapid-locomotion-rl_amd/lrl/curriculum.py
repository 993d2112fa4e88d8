"""Grid-adaptive command curriculum (host side, numpy) — bit-exact with the reference.

Restates ``Curriculum`` / ``RewardThresholdCurriculum`` (mini_gym/envs/base/curriculum.py:16-124):
a 3-D grid of command bins (lin_vel_x, lin_vel_y, ang_vel_yaw) with sampling weights, sampled with
``np.random.RandomState`` (MT19937) so that ``sample``/``update`` reproduce the reference's draws
bit for bit for the same seed.  This is bookkeeping on a few thousand bins once per resampling
interval; it stays on the host like the reference.
"""
import numpy as np


class GridCurriculum:
    """Curriculum (curriculum.py:16-68)."""

    def __init__(self, seed, **key_ranges):
        self.rng = np.random.RandomState(seed)
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
        order, i.e. exactly the per-row calls of curriculum.py:66-68 (np.stack over rows) in sequence."""
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
        self.weights[bin_inds[ok]] = np.clip(self.weights[bin_inds[ok]] + 0.2, 0, 1)
        centres = bin_inds[ok]
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
