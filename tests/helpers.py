"""Shared test helpers: configs, fixture loading, oracle state set-up."""
import os

import numpy as np

from lrl import config as lcfg
from lrl import params as lparams
from lrl.robot import load_robot

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
ROBOT_FILES = {"mc": "mini_cheetah.urdf", "go1": "go1.urdf"}


def make(robot="mc", **over):
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    for k, v in over.items():
        node = cfg
        *ps, leaf = k.split(".")
        for p in ps:
            node = getattr(node, p)
        setattr(node, leaf, v)
    rob = load_robot(ROBOT_FILES[robot])
    if robot == "mc":
        cfg.terrain.x_offset = 0
    P = lparams.build_params(cfg, rob)
    M = lparams.build_model(rob)
    return cfg, rob, M, P


def make_rough(robot="go1", border_size=2.0, **over):
    """Rough-terrain variant of ``make``: trimesh ground, height scan (17 x 11 points -> 42 + 187 obs), terrain
    curriculum; the params carry terrain_mesh = 1 (contacts against lrl_sim_set_terrain's / the oracle's mesh)."""
    over = dict({"terrain.mesh_type": "trimesh", "terrain.measure_heights": True, "terrain.curriculum": True,
                 "terrain.border_size": border_size, "terrain.teleport_robots": False,
                 "env.num_observations": 42 + 187}, **over)
    cfg = lcfg.make_cfg()
    (lcfg.config_mini_cheetah if robot == "mc" else lcfg.config_go1)(cfg)
    for k, v in over.items():
        node = cfg
        *ps, leaf = k.split(".")
        for p in ps:
            node = getattr(node, p)
        setattr(node, leaf, v)
    cfg.terrain.x_offset = 0
    rob = load_robot(ROBOT_FILES[robot])
    P = lparams.build_params(cfg, rob, terrain_mesh=1)
    M = lparams.build_model(rob)
    return cfg, rob, M, P


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
