"""How far the contact model's sphere stand-ins for the URDF mesh colliders are from the meshes (IN-CONTAINER ONLY:
reads the meshes under /root/reference/resources).  PhysX collides a mesh as its convex hull, and against the ground
plane (normal n) a convex body touches first at its support point in direction -n, so the quantity that decides
ground contact is the support function h(d) = max_x x.d.  For every stand-in this prints, over 2,000 directions
spread over the sphere (and over the lower hemisphere of the link frame alone), the largest and mean |h_hull(d) -
h_spheres(d)|, where h_spheres(d) = max_i (c_i.d + r_i) over the stand-in's spheres.  Since round 6 the ground contacts use the support
tables instead (lrl/robot.py support_table, lrl/robots/mini_cheetah_hulls.npz): "table_*" is the same measure for
h_table(d) = the table point's x.d (the max over the mesh's tables: the calf's two halves), over 200,000 random
directions, against the hull of the mesh as the URDF places it in the link frame.
usage: python scripts/mesh_standin_error.py > profiles/<tag>_mesh_support_error.json"""
import json
import os
import sys

import numpy as np
from scipy.spatial import ConvexHull

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
from lrl.robot import _mesh_vertices, _shape_spheres, hull_support, load_robot, rpy_to_mat  # noqa: E402

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
ROB = load_robot("mini_cheetah.urdf")
RNG = np.random.default_rng(0).normal(size=(200000, 3))
RNG /= np.linalg.norm(RNG, axis=1, keepdims=True)
# FR ab/ad (leg 1, body 4) and its calf (body 6), as CASES places them: their tables
TABLES = {"mini_lower_link.obj": sorted({ROB["sphere_hull"][s] for s in range(ROB["num_spheres"])
                                         if ROB["sphere_body"][s] == 6}),
          "mini_abad.obj": sorted({ROB["sphere_hull"][s] for s in range(ROB["num_spheres"]) if ROB["sphere_body"][s] == 4})}
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
    hs = TABLES[fn]
    h_exact = (hv @ RNG.T).max(0)
    h_tab = np.max([np.einsum("nk,nk->n", hull_support(ROB["hull_table"][h], RNG, ROB["hull_res"]), RNG) for h in hs], 0)
    et = h_tab - h_exact
    out[fn].update({"tables": hs, "table_res": ROB["hull_res"], "table_k": ROB["hull_k"],
                    "table_max_abs_mm": round(float(np.abs(et).max() * 1e3), 3),
                    "table_mean_abs_mm": round(float(np.abs(et).mean() * 1e3), 4),
                    "table_max_over_mm": round(float(et.max() * 1e3), 4),
                    "table_lower_hemisphere_max_abs_mm": round(float(np.abs(et[RNG[:, 2] < 0]).max() * 1e3), 3)})
print(json.dumps(out, indent=1))
