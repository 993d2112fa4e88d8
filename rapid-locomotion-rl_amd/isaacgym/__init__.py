"""Import-only stand-in for NVIDIA Isaac Gym (``isaacgym``, Preview 3: proprietary, not vendored in the reference).

The reference's scripts import it first of all (``import isaacgym; assert isaacgym`` — scripts/train.py:3-4,
scripts/test.py:1-3, scripts/play.py:1-3) because Isaac Gym must be imported before torch.  Here the simulator is the
native HIP env kernel behind ``lrl.env`` (liblrl.so), so the package only has to resolve: ``torch_utils`` restates the
tensor helpers mini_gym uses (legged_robot.py:8, math_utils.py:7), ``terrain_utils`` re-exports the height-field
primitives ``lrl.terrain`` restates (terrain.py:6), and ``gymapi`` / ``gymtorch`` / ``gymutil`` hold the few names the
reference touches outside the simulator calls the native library replaces.
"""
from . import gymapi, gymtorch, gymutil, terrain_utils, torch_utils  # noqa: F401
