"""PGS vs TGS on fixed contact scenarios (CPU, the fp64 oracle): the simulator runs velocity-level projected
Gauss-Seidel (solver_iterations sweeps over each 5 ms sub-step, warm-started), while the reference configures PhysX's
TGS solver (legged_robot_config.py:247 solver_type = 1, num_position_iterations 4).  PhysX is closed, so this measures
the gap against a restatement of the TGS scheme in the oracle (lrl_oracle.c lrlo_set_solver_tgs: the sub-step split
into 4 sub-iterations whose targets come from separations moved by the motion so far, positions integrating the
sub-iterations' motion), on the same robot, inputs and contact model:
  stand  — 32 Mini Cheetahs from the default pose, zero actions (PD holding the default pose), 2 s
  drop   — the same from 15 cm higher, 1 s (impact)
  gait   — the reference run's trained policy (tests/golden/checkpoint_last.npz, student act: adaptation module +
           actor) tracking 1 m/s for 3 s after 0.4 s of zero actions
usage: python scripts/tgs_vs_pgs.py > profiles/r4_tgs_vs_pgs.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrl import _abi  # noqa: E402
from lrl import config as lcfg  # noqa: E402
from lrl import params as lparams  # noqa: E402
from lrl.ppo.actor_critic import ActorCritic  # noqa: E402
from lrl.robot import load_robot  # noqa: E402
from oracle import oracle  # noqa: E402

N = 32


def setup():
    cfg = lcfg.make_cfg()
    lcfg.config_mini_cheetah(cfg)
    cfg.terrain.x_offset = 0
    cfg.noise.add_noise = False
    rob = load_robot("mini_cheetah.urdf")
    P, M = lparams.build_params(cfg, rob, solver_type=0), lparams.build_model(rob)  # the study's switch picks the solver
    P.teleport = 0
    return cfg, P, M


def state(P, M, dz=0.0, seed=0):
    st = oracle.make_state(N, M.num_bodies, P.num_obs, P.num_history, P.num_sum_keys + 1, P.num_sum_keys + 5)
    rng = np.random.default_rng(seed)
    st["root"][:, :13] = np.array(P.base_init_state[:], np.float32)
    st["root"][:, 0] = np.arange(N) * 3.0
    st["root"][:, 2] += dz
    st["dof_pos"][:] = np.array(P.default_dof_pos[:], np.float32)
    st["friction"][:] = rng.uniform(0.5, 1.25, N).astype(np.float32)
    st["restitution"][:] = 0.0
    st["commands"][:, 0] = 1.0
    return st


def policy(cfg):
    ac = ActorCritic(cfg.env.num_observations, cfg.env.num_privileged_obs,
                     cfg.env.num_observations * cfg.env.num_observation_history, cfg.env.num_actions)
    g = np.load(os.path.join(ROOT, "tests", "golden", "checkpoint_last.npz"), allow_pickle=False)
    ac.load_state_dict({k: torch.from_numpy(g["sd/" + k]) for k in g["keys"]}, strict=True)
    ac.eval()
    return lambda st: ac.act_student(torch.from_numpy(st["obs"]), torch.from_numpy(st["hist"])).detach().numpy()


def run(P, M, st, steps, pol=None, warm=0):
    flags = _abi.STEP_PHYSICS | _abi.STEP_HISTORY
    feet = list(P.feet[:P.num_feet])
    weight = (M.base_mass + sum(sum(l[:]) for l in M.link_mass)) * 9.81
    h, fz, vx, up = [], [], [], []
    for s in range(steps):
        act = np.zeros((N, 12), np.float32) if (pol is None or s < warm) else pol(st)
        oracle.env_step(M, P, st, act, flags, common_step_counter=s + 1)
        h.append(st["root"][:, 2].copy())
        fz.append(st["contact"][:, feet, 2].sum(1) / weight)
        vx.append(st["base_lin_vel"][:, 0].copy())
        up.append(st["projected_gravity"][:, 2] < -0.8)
    return np.array(h), np.array(fz), np.array(vx), np.array(up)


def main():
    cfg, P, M = setup()
    out = {"envs": N, "dt_policy": float(P.dt), "solver_iterations": int(P.solver_iterations)}
    pol = policy(cfg)
    scen = {"stand": dict(dz=0.0, steps=100), "drop": dict(dz=0.15, steps=50),
            "gait": dict(dz=0.0, steps=170, pol=pol, warm=20)}
    for name, sc in scen.items():
        res = {}
        for tgs in (0, 1):
            oracle.set_solver_tgs(tgs)
            st = state(P, M, sc["dz"])
            h, fz, vx, up = run(P, M, st, sc["steps"], sc.get("pol"), sc.get("warm", 0))
            tail = slice(len(h) // 2, None)
            res["tgs" if tgs else "pgs"] = dict(
                base_height_end=float(h[-1].mean()), base_height_min=float(h.min()),
                foot_force_over_weight_tail=float(fz[tail].mean()), peak_foot_force_over_weight=float(fz.max()),
                fwd_vel_tail=float(vx[tail].mean()), upright_end=float(up[-1].mean()),
                _h=h, _vx=vx)
        oracle.set_solver_tgs(0)
        a, b = res["pgs"], res["tgs"]
        res["diff"] = dict(base_height_max_abs=float(np.abs(a["_h"] - b["_h"]).max()),
                           base_height_rms=float(np.sqrt(((a["_h"] - b["_h"]) ** 2).mean())),
                           fwd_vel_tail_mean=float(a["fwd_vel_tail"] - b["fwd_vel_tail"]))
        for k in ("pgs", "tgs"):
            res[k] = {kk: round(v, 5) for kk, v in res[k].items() if not kk.startswith("_")}
        res["diff"] = {k: round(v, 5) for k, v in res["diff"].items()}
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
