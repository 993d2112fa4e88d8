"""Host curriculum vs the reference's RewardThresholdCurriculum (golden vectors) — bit-exact."""
import numpy as np

from helpers import golden
from lrl.curriculum import RewardThresholdCurriculum


def test_curriculum_bit_exact():
    g = golden("curriculum.npz")
    c = RewardThresholdCurriculum(seed=100, x_vel=(-10.0, 10.0, 51), y_vel=(-0.6, 0.6, 2), yaw_vel=(-10.0, 10.0, 51))
    assert len(c) == 5202 and c._raw_grid.shape == (3, 51, 2, 51)
    np.testing.assert_array_equal(c.grid, g["grid"])
    c.set_to(low=np.array([-0.6, -0.6, -1.0]), high=np.array([0.6, 0.6, 1.0]))
    np.testing.assert_array_equal(c.weights, g["weights0"])
    assert int((c.weights > 0).sum()) == 30  # command_area 0.006 at it 0 (outputs.log:502)
    cmds, bins = c.sample(batch_size=64)
    np.testing.assert_array_equal(bins, g["bins1"])
    np.testing.assert_array_equal(cmds, g["cmds1"])
    c.update(g["upd_bins"], g["lin"], g["ang"], float(g["lin_thr"]), float(g["ang_thr"]), local_range=0.5)
    np.testing.assert_array_equal(c.weights, g["weights1"])
    cmds, bins = c.sample(batch_size=4096)
    np.testing.assert_array_equal(bins, g["bins2"])
    np.testing.assert_array_equal(cmds, g["cmds2"])


def test_curriculum_shape_kat():
    # curriculum.py:127-130 known-answer check
    r = RewardThresholdCurriculum(100, x=(-1, 1, 5), y=(-1, 1, 2), z=(-1, 1, 11))
    assert r._raw_grid.shape == (3, 5, 2, 11)


def test_vectorised_update_equals_the_reference_loop():
    """RewardThresholdCurriculum.update (counted neighbourhood adds) against curriculum.py:105-115 as written
    (_update_literal): identical weights and episode rewards, element for element, over random update sequences —
    duplicate bins, bins at the grid edges, weights near the clip, several local ranges."""
    import copy
    from lrl.curriculum import RewardThresholdCurriculum
    rng = np.random.default_rng(11)
    for trial in range(12):
        c = RewardThresholdCurriculum(seed=100, x_vel=(-10, 10, 51), y_vel=(-0.6, 0.6, 2), yaw_vel=(-10, 10, 51))
        c.weights[:] = rng.choice([0.0, 0.2, 0.6, 0.8, 1.0], len(c)) * (rng.random(len(c)) < 0.5)
        ref = copy.deepcopy(c)
        for step in range(6):
            n = int(rng.integers(1, 300))
            bins = rng.integers(0, len(c), n)
            if step % 2:
                bins[: n // 3] = bins[0]  # duplicates
                bins[-3:] = [0, len(c) - 1, 51 * 2 - 1]
            lin = rng.random(n).astype(np.float32)
            ang = rng.random(n).astype(np.float32)
            lr = [0.5, 0.1, 1.0][trial % 3]
            c.update(bins, lin, ang, 0.3, 0.2, local_range=lr)
            ref._update_literal(bins, lin, ang, 0.3, 0.2, local_range=lr)
            np.testing.assert_array_equal(c.weights, ref.weights)
            np.testing.assert_array_equal(c.episode_reward_lin, ref.episode_reward_lin)
            np.testing.assert_array_equal(c.episode_reward_ang, ref.episode_reward_ang)


def test_native_curriculum_matches_numpy_form():
    """lrl_curriculum_sample / lrl_curriculum_update_weights (csrc/lrl_curriculum.cpp: MT19937, numpy's pairwise sum,
    choice's cdf + searchsorted, the uniform cell draws, the clipped neighbourhood adds) against the numpy form of
    lrl/curriculum.py on the same generator state: identical bins, commands, weights and generator position over random
    update / sample sequences (batch sizes 1 .. 4096, duplicate centres, grid edges, weights at the clip), with draws
    made through ``rng`` in between (the native stream continues from them)."""
    import ctypes as C
    from lrl import _abi
    from lrl.curriculum import RewardThresholdCurriculum
    rng = np.random.default_rng(5)
    L = _abi.lib()
    for n in (1, 7, 8, 127, 128, 129, 1000, 5202, 6001):  # numpy's np.sum restated (pairwise blocks of 8 / 128)
        a = rng.random(n) * rng.choice([1.0, 1e-3, 1e3], n)
        assert L.lrl_np_sum_f64(a.ctypes.data_as(C.c_void_p), n) == np.sum(a)
    for trial in range(6):
        nat = RewardThresholdCurriculum(seed=100 + trial, x_vel=(-10, 10, 51), y_vel=(-0.6, 0.6, 2), yaw_vel=(-10, 10, 51))
        ref = RewardThresholdCurriculum(seed=100 + trial, x_vel=(-10, 10, 51), y_vel=(-0.6, 0.6, 2), yaw_vel=(-10, 10, 51))
        assert nat._native
        ref._native = False  # the numpy form
        for c in (nat, ref):
            c.set_to(low=np.array([-1.0, -0.6, -1.0]), high=np.array([1.0, 0.6, 1.0]))
        for step in range(8):
            n = int(rng.choice([1, 3, 64, 500, 4096]))
            cn, bn = nat.sample(n)
            cr, br = ref.sample(n)
            np.testing.assert_array_equal(bn, br)
            np.testing.assert_array_equal(cn, cr)
            lin = rng.random(n).astype(np.float32)
            ang = rng.random(n).astype(np.float32)
            bins = bn.copy()
            if step % 3 == 1:
                bins[: n // 2] = bins[0]
                bins[-1:] = len(nat) - 1
            nat.update(bins, lin, ang, 0.3, 0.2, local_range=[0.5, 0.1, 1.0][step % 3])
            ref.update(bins, lin, ang, 0.3, 0.2, local_range=[0.5, 0.1, 1.0][step % 3])
            np.testing.assert_array_equal(nat.weights, ref.weights)
            if step == 4:  # a draw through the RandomState view: both streams continue from it
                assert nat.rng.random_sample() == ref.rng.random_sample()
            if step == 5:  # a deep copy continues the same stream on its own arrays (no shared native caches)
                import copy
                twin = copy.deepcopy(nat)
                np.testing.assert_array_equal(twin.sample(9)[1], copy.deepcopy(nat).sample(9)[1])
                assert twin.weights is not nat.weights
        assert nat.rng.get_state()[2] == ref.rng.get_state()[2]
        np.testing.assert_array_equal(nat.rng.get_state()[1], ref.rng.get_state()[1])
