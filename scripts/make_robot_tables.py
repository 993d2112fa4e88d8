"""Tabulate the reference's robot assets into rapid-locomotion-rl_amd/lrl/robots/*.json.

IN-CONTAINER ONLY (reads the URDFs/meshes under /root/reference/resources, which are not on the
GPU box).  The tables hold derived model data (masses, inertias, joint frames, collision spheres, the mesh
colliders' hull vertex sets and support tables in <name>_hulls.npz), not reference source.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
from lrl.robot import build_quadruped, support_table  # noqa: E402

SRC = {
    "mini_cheetah": "/root/reference/resources/robots/mini_cheetah/urdf/mini_cheetah.urdf",
    "go1": "/root/reference/resources/robots/go1/urdf/go1.urdf",
}
for name, path in SRC.items():
    m = build_quadruped(path)
    m["source"] = os.path.relpath(path, "/root/reference")
    hv = m.pop("hull_vertices")
    if hv:  # mesh colliders: support tables + the hull vertex sets they were built from, beside the table
        m["hull_file"] = name + "_hulls.npz"
        arrs = {"tables": np.stack([support_table(np.asarray(v)) for v in hv])}
        arrs.update({"verts_%d" % h: np.asarray(v) for h, v in enumerate(hv)})
        np.savez_compressed(os.path.join(ROOT, "rapid-locomotion-rl_amd", "lrl", "robots", m["hull_file"]), **arrs)
    out = os.path.join(ROOT, "rapid-locomotion-rl_amd", "lrl", "robots", name + ".json")
    with open(out, "w") as f:
        json.dump(m, f, indent=1)
    print(name, "bodies", m["body_names"], "spheres", m["num_spheres"], "mass",
          m["base_mass"] + sum(sum(x) for x in m["link_mass"]))
