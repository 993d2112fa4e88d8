"""mini_gym/utils/terrain.py surface."""
from lrl.terrain import Terrain  # noqa: F401
