"""Tabulate the reference's robot assets into rapid-locomotion-rl_amd/lrl/robots/*.json.

IN-CONTAINER ONLY (reads the URDFs/meshes under /root/reference/resources, which are not on the
GPU box).  The tables hold derived model data (masses, inertias, joint frames, collision spheres),
not reference source.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
from lrl.robot import build_quadruped  # noqa: E402

SRC = {
    "mini_cheetah": "/root/reference/resources/robots/mini_cheetah/urdf/mini_cheetah.urdf",
    "go1": "/root/reference/resources/robots/go1/urdf/go1.urdf",
}
for name, path in SRC.items():
    m = build_quadruped(path)
    m["source"] = os.path.relpath(path, "/root/reference")
    out = os.path.join(ROOT, "rapid-locomotion-rl_amd", "lrl", "robots", name + ".json")
    with open(out, "w") as f:
        json.dump(m, f, indent=1)
    print(name, "bodies", m["body_names"], "spheres", m["num_spheres"], "mass",
          m["base_mass"] + sum(sum(x) for x in m["link_mass"]))
