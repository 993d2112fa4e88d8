"""lrl — MI355X-native legged-locomotion hot path (LeggedRobot.step + PPO numerics).

Host-side mirror of the reference's env / PPO surfaces over the C-ABI library liblrl.so
(include/lrl.h).  See DESIGN.md.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)
