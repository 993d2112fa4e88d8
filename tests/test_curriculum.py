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
