"""Diagnostic for a physics-parity outlier (tests/test_env_gpu.py::_physics_vs_oracle): replays the test's states for
``robot n steps`` and, for every env outside tolerance, re-runs that env alone in the oracle from 32 fp32-size
perturbations of its start state, to tell an oracle-sensitive env (the kernel's result inside the perturbed spread)
from a kernel defect (outside it).  usage: python scripts/tgs_probe.py mc 4096 10 [solver_type]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "rapid-locomotion-rl_amd"), ROOT]
import numpy as np  # noqa: E402

import test_env_gpu as T  # noqa: E402
from helpers import SEP_EPS_1, make, perturb_state, physics_mismatch, within_tolerance  # noqa: E402
from lrl import _abi  # noqa: E402
from oracle import oracle  # noqa: E402

FIELDS = ("root", "dof_pos", "dof_vel", "contact")


def one(st, e):
    return {k: (v[:, e:e + 1] if k in ("episode_sums", "command_sums") else v[e:e + 1]).copy() for k, v in st.items()}


def main():
    robot, n, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    over = {} if len(sys.argv) < 5 else {"sim.physx.solver_type": int(sys.argv[4])}
    cfg, rob, M, P = make(robot, **{"env.num_envs": n}, **over)
    env = T._env(robot, n, **over)
    rng = np.random.default_rng(5 + steps)
    root, dof, dofv = T._random_states(rng, n, P, robot)
    st = oracle.make_state(n, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
    fr = rng.uniform(0.05, 4.5, n).astype(np.float32)
    rs = rng.uniform(0, 1, n).astype(np.float32)
    pl = rng.uniform(-1, 3, n).astype(np.float32)
    com = rng.uniform(-0.1, 0.1, (n, 3)).astype(np.float32)
    for k, v in dict(root=root, dof_pos=dof, dof_vel=dofv, friction=fr, restitution=rs, payload=pl, com=com).items():
        st[k][:] = v
    env.friction_coeffs[:] = T._dev(fr)
    env.restitutions[:] = T._dev(rs)
    env.payloads[:] = T._dev(pl)
    env.com_displacements[:] = T._dev(com)
    flags = _abi.STEP_PHYSICS | _abi.STEP_INJECT_UNIFORM
    rng_p = np.random.default_rng(77)
    for s in range(steps):
        env.root_states[:] = T._dev(st["root"])
        env.dof_pos[:] = T._dev(st["dof_pos"])
        env.dof_vel[:] = T._dev(st["dof_vel"])
        act = (rng.normal(size=(n, 12)) * 0.5).astype(np.float32)
        noise = rng.random((n, P.num_obs)).astype(np.float32)
        dr = rng.random(n).astype(np.float32)
        T._step_raw(env, T._dev(act), flags, T._dev(noise), T._dev(dr))
        st0 = {k: v.copy() for k, v in st.items()}
        st_p = perturb_state(st, rng_p)
        m = np.zeros((n, 2))
        oracle.env_step(M, P, st, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1, margins=m)
        oracle.env_step(M, P, st_p, act, flags, noise_u=noise, dr_u=dr, common_step_counter=s + 1)
        got = {k: T._np(getattr(env, a)) for k, a in dict(root="root_states", dof_pos="dof_pos", dof_vel="dof_vel",
                                                            contact="contact_forces").items()}
        sens = ~within_tolerance(st_p, st)
        bad, excl = physics_mismatch(got, st, m, sens, sep_eps=SEP_EPS_1)
        print(f"step {s + 1}: {bad.sum()} bad, {excl.sum()} excluded", flush=True)
        for e in np.flatnonzero(bad)[:4]:
            kerr = {k: float(np.abs(got[k][e] - st[k][e]).max()) for k in FIELDS}
            spread = {k: 0.0 for k in FIELDS}
            n_out = 0
            g = np.random.default_rng(1000 + e)
            for _ in range(32):
                sp = perturb_state(one(st0, e), g)
                oracle.env_step(M, P, sp, act[e:e + 1], flags, noise_u=noise[e:e + 1], dr_u=dr[e:e + 1],
                                common_step_counter=s + 1)
                for k in FIELDS:
                    spread[k] = max(spread[k], float(np.abs(sp[k][0] - st[k][e]).max()))
                n_out += int(not within_tolerance(sp, one(st, e))[0])
            solo = one(st0, e)
            oracle.env_step(M, P, solo, act[e:e + 1], flags, noise_u=noise[e:e + 1], dr_u=dr[e:e + 1],
                            common_step_counter=s + 1)
            same = all(np.array_equal(solo[k][0], st[k][e]) for k in FIELDS)
            print(f"  env {e}: kernel err {kerr}\n    oracle spread over 32 perturbations {spread} "
                  f"({n_out}/32 outside tolerance; solo replay identical: {same}); margins {m[e]}", flush=True)
            diff = np.abs(got["dof_vel"][e] - st["dof_vel"][e])
            print("    dof_vel kernel", np.round(got["dof_vel"][e], 4).tolist(), "\n    dof_vel oracle",
                  np.round(st["dof_vel"][e], 4).tolist(), "worst joint", int(diff.argmax()), flush=True)
            print("    contact z kernel", np.round(got["contact"][e][:, 2], 3).tolist(), "\n    contact z oracle",
                  np.round(st["contact"][e][:, 2], 3).tolist(), flush=True)
        if bad.any() and s >= 1:
            break
    env.close()


if __name__ == "__main__":
    main()
