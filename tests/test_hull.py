"""Leg colliders as support tables (CPU): the Mini Cheetah's ab/ad and calf meshes, which PhysX collides as their convex
hulls (mini_cheetah.urdf:119-124, 176-181), and the rod boxes of both presets' thighs / calves meet the plane at the
support point a cube-map table gives (lrl/robot.py support_table).  Checked here: the tables reproduce each hull's support function within 1 mm, the
oracle's lookup (lrl_oracle.c hull_support) picks the table's point, the model carries the tables through the C ABI,
and (in this container only) the committed tables are the ones the builder makes from the reference's meshes."""
import ctypes as C
import os

import numpy as np
import pytest

from lrl import params as lparams
from lrl.robot import hull_support, load_robot, support_cell, support_table
from oracle import oracle as O


def _dirs(n, seed=0):
    d = np.random.default_rng(seed).normal(size=(n, 3))
    return d / np.linalg.norm(d, axis=1, keepdims=True)


def _mesh_groups(rob):
    """sphere body -> its support tables (one per stand-in sphere of the body's mesh)"""
    out = {}
    for s, h in enumerate(rob["sphere_hull"]):
        if h >= 0:
            out.setdefault(rob["sphere_body"][s], []).append(h)
    return out


def test_leg_meshes_and_rod_boxes_have_support_tables():
    """Mini Cheetah: the ab/ad mesh (one table), the thigh's rod box and the calf mesh (the two halves of their capsule
    stand-ins); Go1: the thigh and calf rod boxes.  Spheres, the capsules of the URDF cylinders (the presets'
    replace_cylinder_with_capsule, legged_robot_config.py:133) and the base box's corners stay exact as they are."""
    legs = ("FL", "FR", "RL", "RR")
    for urdf, parts in (("mini_cheetah.urdf", {"hip": 1, "thigh": 2, "calf": 2}), ("go1.urdf", {"thigh": 2, "calf": 2})):
        rob = load_robot(urdf)
        g = _mesh_groups(rob)
        names = {rob["body_names"][b]: len(hs) for b, hs in g.items()}
        assert names == {f"{l}_{k}": c for l in legs for k, c in parts.items()}, urdf
        assert rob["hull_table"].shape == (rob["num_hulls"], 6 * rob["hull_res"] ** 2, rob["hull_k"], 4)
        assert rob["hull_k"] == 4


@pytest.mark.parametrize("urdf", ["mini_cheetah.urdf", "go1.urdf"])
def test_support_tables_within_1mm_of_the_hulls(urdf):
    """max over 200k random directions of h_hull(d) - h_table(d), per collider (the calf: the max over its two halves),
    and the table never reaches past the hull (its points are hull vertices)"""
    rob = load_robot(urdf)
    D = _dirs(200_000)
    for b, hs in _mesh_groups(rob).items():
        V = np.concatenate([rob["hull_vertices"][h] for h in hs])
        exact = (V @ D.T).max(0)
        tab = np.max([np.einsum("nk,nk->n", hull_support(rob["hull_table"][h], D, rob["hull_res"]), D) for h in hs], 0)
        err = exact - tab
        assert err.max() < 1.0e-3, (rob["body_names"][b], err.max())
        assert err.min() > -1e-6
        for h in hs:  # every candidate is a vertex of its part
            tv = rob["hull_table"][h][..., :3].reshape(-1, 3).astype(np.float64)
            hv = rob["hull_vertices"][h]
            dist = np.min(np.linalg.norm(tv[:, None, :] - hv[None, :, :], axis=-1), axis=1)
            assert dist.max() < 1e-6


def test_support_cell_rule():
    """major axis with the x, y, z tie order, faces, clamped edges"""
    N = 16
    assert support_cell([1.0, 0.0, 0.0], N) == (0 * N + 8) * N + 8
    assert support_cell([-1.0, 0.0, 0.0], N) == (1 * N + 8) * N + 8
    assert support_cell([0.0, 0.0, -1.0], N) == (5 * N + 8) * N + 8
    assert support_cell([1.0, 1.0, 0.0], N) == (0 * N + 15) * N + 8  # tie |x| = |y| -> x; u = 1 clamps to N - 1
    assert support_cell([0.0, 1.0, 1.0], N) == (2 * N + 15) * N + 8  # tie |y| = |z| -> y; u = z / |y| = 1
    assert support_cell([0.5, -1.0, 0.0], N) == (3 * N + 8) * N + 12  # face -y: u = z = 0, v = x / 1 = 0.5
    t = support_table(np.eye(3), N=2, K=4)
    assert t.shape == (24, 4, 4)


def test_oracle_lookup_matches_the_table():
    """lrlo_hull_support (the oracle's lookup, fp64) returns the table point numpy's hull_support picks"""
    rob = load_robot("mini_cheetah.urdf")
    M = lparams.build_model(rob)
    L = O.lib()
    f = L.lrlo_hull_support
    f.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    f.restype = None
    D = _dirs(3000, seed=1)
    out = np.zeros(3)
    for h in range(rob["num_hulls"]):
        want = hull_support(rob["hull_table"][h], D, rob["hull_res"])
        for i in range(len(D)):
            d = np.ascontiguousarray(D[i])
            f(C.addressof(M), h, d.ctypes.data_as(C.POINTER(C.c_double)), out.ctypes.data_as(C.POINTER(C.c_double)))
            assert np.array_equal(out, want[i]), (h, i)


def test_model_carries_the_tables():
    rob = load_robot("mini_cheetah.urdf")
    M = lparams.build_model(rob)
    assert M.num_hulls == rob["num_hulls"] and M.hull_res == rob["hull_res"] and M.hull_k == 4
    assert list(M.sphere_hull)[:rob["num_spheres"]] == rob["sphere_hull"]
    n = rob["num_hulls"] * 6 * rob["hull_res"] ** 2 * 4 * 4
    got = np.ctypeslib.as_array(C.cast(M.hull_table, C.POINTER(C.c_float)), (n,))
    assert np.array_equal(got, rob["hull_table"].ravel())


def test_straight_down_support_point():
    """straight down (the standing robot's foot contact): each table's point is its part's lowest vertex"""
    rob = load_robot("mini_cheetah.urdf")
    D = np.array([[0.0, 0.0, -1.0]])
    for h in {rob["sphere_hull"][s] for s in range(rob["num_spheres"]) if rob["sphere_hull"][s] >= 0}:
        p = hull_support(rob["hull_table"][h], D, rob["hull_res"])[0]
        exact = rob["hull_vertices"][h][:, 2].min()
        assert abs(p[2] - exact) < 1e-3


@pytest.mark.skipif(not os.path.isdir("/root/reference/resources/robots/mini_cheetah"),
                    reason="reference meshes only in the build container")
def test_committed_tables_are_the_builders():
    """scripts/make_robot_tables.py's tables from the reference meshes equal the committed .npz"""
    from lrl.robot import build_quadruped
    m = build_quadruped("/root/reference/resources/robots/mini_cheetah/urdf/mini_cheetah.urdf")
    rob = load_robot("mini_cheetah.urdf")
    assert m["sphere_hull"] == rob["sphere_hull"]
    for h, v in enumerate(m["hull_vertices"]):
        assert np.array_equal(np.asarray(v), rob["hull_vertices"][h])
    for h in (0, 3):  # (the FL ab/ad and calf-top tables: the greedy build takes a few seconds each)
        assert np.array_equal(support_table(np.asarray(m["hull_vertices"][h])), rob["hull_table"][h])
