"""Rough-terrain generation (lrl/terrain.py) against the reference's Terrain class (mini_gym/utils/terrain.py,
run over the same terrain_utils restatement: tests/golden/terrain.npz) — bit-exact layout, tile types and
env origins — plus structural properties of the primitives (parity unpinned: isaacgym.terrain_utils is not
vendored)."""
import types

import numpy as np

from helpers import golden
from lrl import terrain as T


def _cfg(**kw):
    c = types.SimpleNamespace(mesh_type="trimesh", curriculum=True, selected=False, terrain_kwargs=None,
                              terrain_proportions=[0.1] * 10, num_rows=3, num_cols=10, terrain_length=8.0,
                              terrain_width=8.0, horizontal_scale=0.1, vertical_scale=0.005, border_size=2.0,
                              difficulty_scale=1.0, max_platform_height=0.2, terrain_smoothness=0.005,
                              terrain_noise_magnitude=0.1, slope_treshold=0.75)
    c.__dict__.update(kw)
    return c


def test_terrain_matches_reference_layout():
    g = golden("terrain.npz")
    for name, kw in (("curriculum", {}), ("random", dict(curriculum=False, num_rows=2, num_cols=3))):
        np.random.seed(int(g[name + "_seed"]))
        c = _cfg(**kw)
        t = T.Terrain(c, 64)
        np.testing.assert_array_equal(t.height_field_raw, g[name + "_hf"])
        np.testing.assert_array_equal(c.env_origins, g[name + "_origins"])
        if name == "curriculum":
            assert len(t.triangles) == int(g["curriculum_ntri"])
            np.testing.assert_allclose(t.vertices.astype(np.float64).sum(0), g["curriculum_vsum"], rtol=1e-9)


def test_primitives_structure():
    sub = lambda: T.SubTerrain(width=80, length=80, vertical_scale=0.005, horizontal_scale=0.1)
    t = T.pyramid_stairs_terrain(sub(), step_width=0.31, step_height=0.1, platform_size=3.0)
    hf = t.height_field_raw
    assert hf[0, 0] == 0 and hf[40, 40] == hf.max() and np.all(np.diff(hf[40, :40]) >= 0)
    assert set(np.unique(hf)) <= set(range(0, hf.max() + 1, 20))  # steps of 0.1 m = 20 units
    t = T.pyramid_sloped_terrain(sub(), slope=0.2, platform_size=3.0)
    assert t.height_field_raw[40, 40] == t.height_field_raw.max() and t.height_field_raw[0, 0] == 0
    np.random.seed(0)
    t = T.random_uniform_terrain(sub(), min_height=-0.05, max_height=0.05, step=0.005, downsampled_scale=0.2)
    assert np.abs(t.height_field_raw).max() <= 10
    np.random.seed(0)
    t = T.stepping_stones_terrain(sub(), stone_size=1.0, stone_distance=0.1, max_height=0.0, platform_size=4.0)
    assert t.height_field_raw.min() == int(-10 / 0.005) and t.height_field_raw[40, 40] == 0
    v, tri = T.convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
    assert v.shape == (80 * 80, 3) and tri.shape == (2 * 79 * 79, 3) and tri.max() == 80 * 80 - 1
