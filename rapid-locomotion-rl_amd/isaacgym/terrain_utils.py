"""``isaacgym.terrain_utils`` as mini_gym/utils/terrain.py calls it (SubTerrain and the height-field primitives,
convert_heightfield_to_trimesh): the restatements in ``lrl.terrain`` (parity unpinned: not vendored)."""
from lrl.terrain import (SubTerrain, convert_heightfield_to_trimesh, discrete_obstacles_terrain,  # noqa: F401
                         pyramid_sloped_terrain, pyramid_stairs_terrain, random_uniform_terrain,
                         stepping_stones_terrain)
