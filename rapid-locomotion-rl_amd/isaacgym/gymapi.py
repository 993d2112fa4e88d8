"""``isaacgym.gymapi``: the simulator API the native library replaces (lrl_sim_* in include/lrl.h).
Importable so the reference's modules resolve; acquiring the PhysX simulator itself is refused."""
from dataclasses import dataclass

UP_AXIS_Z = 1
SIM_PHYSX = 1


@dataclass
class Vec3:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0


def acquire_gym():
    raise NotImplementedError("PhysX is not part of this framework: the env step runs in liblrl.so "
                              "(lrl.env.VelocityTrackingEasyEnv)")
