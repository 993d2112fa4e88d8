"""Debug aid: rerun one physics-parity case of tests/test_env_gpu.py and print, for the envs outside tolerance,
which outputs differ and by how much, and how close their joints came to the URDF limits.
usage: python scripts/physics_debug.py mc 256 10 [limits] [nolimits]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "rapid-locomotion-rl_amd"), ROOT]
import numpy as np  # noqa: E402

import test_env_gpu as T  # noqa: E402
from helpers import within_tolerance  # noqa: E402

robot, n, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
limits = "limits" in sys.argv[4:]
if "nolimits" in sys.argv[4:]:  # both sides without the joint-limit rows
    import functools
    from lrl import params as lparams
    lparams.build_params = functools.partial(lparams.build_params, joint_limits=False)
orig = T.physics_mismatch
cap = {}


def spy(got, st, margins, sens=None):
    cap.update(got=got, st=st, margins=margins, sens=sens)
    return orig(got, st, margins, sens)


T.physics_mismatch = spy
try:
    got, st, M = T._physics_vs_oracle(robot, n, steps, limits=limits)
except AssertionError as ex:
    print("assertion:", ex)
got, st, margins = cap["got"], cap["st"], cap["margins"]
M = T.make(robot, **{"env.num_envs": n})[2]
ok = within_tolerance(got, st)
lo, hi = np.array(M.dof_lower[:]), np.array(M.dof_upper[:])
for e in np.flatnonzero(~ok)[:12]:
    d = {k: np.abs(got[k][e] - st[k][e]).max() for k in ("dof_pos", "dof_vel", "contact")}
    d["pos"] = np.abs(got["root"][e, :3] - st["root"][e, :3]).max()
    d["quat"] = np.abs(got["root"][e, 3:7] - st["root"][e, 3:7]).max()
    d["vel"] = np.abs(got["root"][e, 7:] - st["root"][e, 7:]).max()
    lim = np.minimum(hi - st["dof_pos"][e], st["dof_pos"][e] - lo)
    print(e, {k: float(f"{v:.3g}") for k, v in d.items()}, "margins", margins[e], "min limit dist",
          float(lim.min()), "z", st["root"][e, 2])
