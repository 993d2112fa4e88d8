"""Drop-in module path for the reference's ``mini_gym`` package: re-exports the
MI355X implementation in ``lrl``."""
import os

MINI_GYM_ROOT_DIR = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))
MINI_GYM_ENVS_DIR = os.path.join(MINI_GYM_ROOT_DIR, "mini_gym", "envs")
