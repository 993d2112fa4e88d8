"""How far the contact model's sphere stand-ins for the URDF mesh colliders are from the meshes (IN-CONTAINER ONLY:
reads the meshes under /root/reference/resources).  PhysX collides a mesh as its convex hull, and against the ground
plane (normal n) a convex body touches first at its support point in direction -n, so the quantity that decides
ground contact is the support function h(d) = max_x x.d.  For every stand-in this prints, over 2,000 directions
spread over the sphere (and over the lower hemisphere of the link frame alone), the largest and mean |h_hull(d) -
h_spheres(d)|, where h_spheres(d) = max_i (c_i.d + r_i) over the stand-in's spheres.
usage: python scripts/mesh_standin_error.py"""
import json
import os
import sys

import numpy as np
from scipy.spatial import ConvexHull

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
from lrl.robot import _mesh_vertices, _shape_spheres, rpy_to_mat  # noqa: E402

MESHES = "/root/reference/resources/robots/mini_cheetah/meshes/"
# (mesh, collision origin rpy, xyz) as mini_cheetah.urdf places them (the calf: :176-181; the FR abad: :119-124)
CASES = [("mini_lower_link.obj", (0.0, 3.141592, 0.0), (0.0, 0.0, 0.0)),
         ("mini_abad.obj", (3.141592, 0.0, 1.5708), (-0.055, 0.0, 0.0))]


def directions(n=2000):
    i = np.arange(n) + 0.5  # Fibonacci sphere
    phi = np.arccos(1 - 2 * i / n)
    th = np.pi * (1 + 5 ** 0.5) * i
    return np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], 1)


out = {}
D = directions()
for fn, rpy, xyz in CASES:
    v = _mesh_vertices(os.path.join(MESHES, fn), (1, 1, 1))
    v = (rpy_to_mat(rpy) @ v.T).T + np.asarray(xyz)
    hv = v[ConvexHull(v).vertices]
    sph = _shape_spheres("aabb", np.eye(4), (v.min(0), v.max(0)))  # the stand-in lrl/robot.py builds
    C = np.array([c for c, _ in sph])
    R = np.array([r for _, r in sph])
    h_hull = (hv @ D.T).max(0)
    h_sph = (C @ D.T + R[:, None]).max(0)
    err = h_sph - h_hull  # > 0: the stand-in reaches further than the mesh in that direction
    low = D[:, 2] < 0
    out[fn] = {"hull_vertices": int(len(hv)), "spheres": [[list(np.round(c, 4)), round(float(r), 4)] for c, r in sph],
               "max_abs_mm": round(float(np.abs(err).max() * 1e3), 2),
               "mean_abs_mm": round(float(np.abs(err).mean() * 1e3), 2),
               "max_over_mm": round(float(err.max() * 1e3), 2), "max_short_mm": round(float(-err.min() * 1e3), 2),
               "lower_hemisphere_max_abs_mm": round(float(np.abs(err[low]).max() * 1e3), 2),
               "straight_down_mm": round(float((h_sph - h_hull)[np.argmin(D[:, 2])] * 1e3), 2)}
print(json.dumps(out, indent=1))
