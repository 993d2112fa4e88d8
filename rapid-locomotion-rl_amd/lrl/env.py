"""Legged-robot vector env over liblrl.so — the reference's env surface, MI355X underneath.

``LeggedRobotEnv`` mirrors ``LeggedRobot`` (mini_gym/envs/base/legged_robot.py) plus the
``VelocityTrackingEasyEnv`` 4-tuple ``step`` (mini_gym/envs/mini_cheetah/velocity_tracking/
velocity_tracking_easy_env.py:42-69): the same constructor arguments, attribute names and
buffers (``root_states``, ``dof_pos``, ``commands``, ``episode_sums``, ``extras`` ...), with every
per-env computation of ``step`` fused into one HIP launch (``lrl_sim_step``).  The torch tensors
exposed here are zero-copy views of the sim's struct-of-arrays HBM buffers, so writes such as
``env.commands[:, 0] = 1.0`` act on the simulation directly (the reference needs a
``set_*_tensor`` call for that; here those calls exist but the data is already in place).

Semantics follow the fork by default (no automatic resets inside ``step``,
commands only written by callers).  Host-side bookkeeping that the reference also does on the
host — the command curriculum (numpy MT19937) and the per-reset episode logging — stays in Python.
"""
import ctypes as C
import math
import os

import numpy as np
import torch

from . import _abi, _dlpack
from . import params as lparams
from .config import Section
from .curriculum import RewardThresholdCurriculum
from .robot import load_robot
from .terrain import Terrain, convert_heightfield_to_trimesh

# Cfg.asset.file is formatted with the package root, as mini_gym does; only its file name selects the robot's
# committed model table (lrl/robots/<name>.json) — no URDF is read at run time
MINI_GYM_ROOT_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_SNAPSHOT_EXTRAS = os.environ.get("LRL_EXTRAS_SNAPSHOT", "1") != "0"


class _LazyExtras(dict):
    """``extras`` dict whose per-step numpy entries (velocity_tracking_easy_env.py:48-62) are step-time snapshots: step
    enqueues one device copy of the fields they read (lrl_sim_extras_snapshot, into a buffer of that step's own), and an
    entry becomes a numpy array only when read (the reference pays 11 device->host syncs per step).  As in the
    reference, ``extras`` is one dict updated by every step, so reading a key after the next step gives the next
    step's values; an array read, or a ``copy()`` / ``dict(...)`` / ``items()`` taken, holds the step it came from."""

    def __init__(self, env):
        super().__init__()
        self._env = env
        self._lazy = {}
        self._cond = {}  # key -> (value, present()): an entry whose presence is decided on first access

    def set_lazy(self, key, fn):
        self._cond.pop(key, None)
        self._lazy[key] = fn
        dict.pop(self, key, None)

    def set_conditional(self, key, value, present):
        """``key`` holds ``value`` if ``present()`` is true when the dict is first asked about it (membership, a read,
        keys()); otherwise the key is absent for this step.  Deciding calls ``present()`` — on the device reset path
        a one-element device->host read, i.e. a stream sync — so ``len(extras)``, ``keys()`` or iteration resolves every
        pending key and pays that sync once per step, where reading only the keys a caller needs does not; the
        reference's Runner tests and reads ``infos["train/episode"]`` by key (mini_gym_learn/ppo/__init__.py:145-147)."""
        self._lazy.pop(key, None)
        dict.pop(self, key, None)
        self._cond[key] = (value, present)

    def _resolve(self, key):
        c = self._cond.pop(key, None)
        if c is not None and c[1]():
            dict.__setitem__(self, key, c[0])

    def _get(self, key):
        self._resolve(key)
        fn = self._lazy.pop(key, None)
        if fn is not None:  # materialise once: later reads return the same array
            dict.__setitem__(self, key, fn())
        return dict.__getitem__(self, key)

    def __getitem__(self, key):
        return self._get(key)

    def __setitem__(self, key, value):
        self._lazy.pop(key, None)
        self._cond.pop(key, None)
        dict.__setitem__(self, key, value)

    def __delitem__(self, key):
        found = self._cond.pop(key, None) is not None
        found = self._lazy.pop(key, None) is not None or found
        if dict.__contains__(self, key):
            dict.__delitem__(self, key)
        elif not found:
            raise KeyError(key)

    def __contains__(self, key):
        self._resolve(key)
        return dict.__contains__(self, key) or key in self._lazy

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self.keys())

    def get(self, key, default=None):
        return self._get(key) if key in self else default

    def pop(self, key, *default):
        if key in self:
            v = self._get(key)
            dict.pop(self, key)
            return v
        if default:
            return default[0]
        raise KeyError(key)

    def keys(self):
        for k in list(self._cond):
            self._resolve(k)
        return list(dict.keys(self)) + [k for k in self._lazy if not dict.__contains__(self, k)]

    def items(self):
        return [(k, self._get(k)) for k in self.keys()]

    def values(self):
        return [self._get(k) for k in self.keys()]

    def copy(self):
        return dict(self.items())

    def update(self, other=(), **kw):
        for k, v in (other.items() if hasattr(other, "items") else other):
            self[k] = v
        for k, v in kw.items():
            self[k] = v


class _Upload:
    """Host -> device staging through pinned buffers: each put() packs numpy arrays into one pinned slot and issues one
    non-blocking copy on the current stream, returning typed device views of it.  A ring of slots, each rewritten only
    after its previous copy ran (an event per slot); the views are for stream-ordered use right away (a slot comes
    round again after len(slots) puts)."""

    _TD = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32, np.dtype(np.float32): torch.float32}

    def __init__(self, device, nbytes, slots=4):
        self.host = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(slots)]
        self.hnp = [h.numpy() for h in self.host]
        self.dev = [torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(slots)]
        self.ev = [torch.cuda.Event() for _ in range(slots)]
        self.used = [False] * slots
        self.i = 0

    def put(self, *arrays):
        i = self.i
        self.i = (i + 1) % len(self.host)
        if self.used[i]:
            self.ev[i].synchronize()
        h, off, spans = self.hnp[i], 0, []
        for a in arrays:
            a = np.ascontiguousarray(a)
            nb = a.nbytes
            h[off:off + nb] = a.reshape(-1).view(np.uint8)
            spans.append((off, nb, a.dtype, a.shape))
            off = (off + nb + 255) // 256 * 256
        if off > h.shape[0]:
            raise ValueError("_Upload: slot too small")
        self.dev[i][:off].copy_(self.host[i][:off], non_blocking=True)
        self.ev[i].record()
        self.used[i] = True
        return [self.dev[i][o:o + nb].view(self._TD[dt]).view(shape) for o, nb, dt, shape in spans]


class LeggedRobotEnv:
    def __init__(self, sim_device="cuda:0", headless=True, num_envs=None, prone=False, deploy=False, cfg=None,
                 eval_cfg=None, initial_dynamics_dict=None, physics_engine="SIM_PHYSX", seed=0, env_offset=None,
                 solver_iterations=None, legacy_fork=True, num_envs_global=None, device_resets=None):
        if cfg is None:
            from .config import Cfg as cfg
        if num_envs is not None:
            cfg.env.num_envs = num_envs
        if prone:  # velocity_tracking_easy_env.py:16-19
            cfg.init_state.rot = [0.0, 1.0, 0.0, 0.0]
            cfg.init_state.pos = [0.0, 0.0, 0.15]
            cfg.asset.fix_base_link = True
        if deploy:
            cfg.noise.add_noise = False
            cfg.domain_rand.push_robots = False
            cfg.domain_rand.randomize_friction = False
            cfg.env.episode_length_s = 100
        self.cfg, self.eval_cfg = cfg, eval_cfg
        # legacy_fork=False re-enables what the fork comments out: reset_idx inside step
        # for terminated / timed-out envs, command resampling every resampling_time and at resets
        self.legacy_fork = bool(legacy_fork)
        # data-parallel ranks: with the upstream curricula reconnected, every rank applies the same
        # command-curriculum update / sample to all ranks' reset envs (rank-major global order), so the replicas of
        # the curriculum stay identical and a rank's envs draw what they would in one process holding every env
        self._dist = None
        if not self.legacy_fork:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                self._dist = dist
        self.device = torch.device(sim_device)
        if self.device.type != "cuda" or not torch.cuda.is_available():
            raise RuntimeError("LeggedRobotEnv runs on the GPU through liblrl.so; no CPU path exists")
        self.headless = True
        # train / eval split (base_task.py:43-50): eval envs follow the train envs in one sim
        self.num_train_envs = cfg.env.num_envs
        self.num_eval_envs = eval_cfg.env.num_envs if eval_cfg is not None else 0
        self.num_envs = self.num_train_envs + self.num_eval_envs
        self.num_obs = cfg.env.num_observations
        self.num_privileged_obs = cfg.env.num_privileged_obs
        self.num_actions = cfg.env.num_actions
        self.seed = int(seed)
        # data-parallel sharding: this sim holds global envs [env_offset, env_offset + num_envs) of
        # num_envs_global.  Every per-env draw is keyed by the global id and the env origins are the global grid's, so
        # a rank's envs evolve exactly as the same envs of one process holding all of them.  Default: equal shards over
        # the initialised process group (the bench's layout: env_offset = rank x num_envs), else env_offset + num_envs.
        import torch.distributed as tdist
        _pg = tdist.is_available() and tdist.is_initialized()
        world = tdist.get_world_size() if _pg else 1
        if env_offset is None:  # (a rank > 0 left at offset 0 would repeat rank 0's draws and origins)
            env_offset = tdist.get_rank() * self.num_envs if _pg else 0
        self.env_offset = int(env_offset)
        if num_envs_global is None:
            num_envs_global = max(self.num_envs * world, self.env_offset + self.num_envs) if self.env_offset or \
                world > 1 else self.num_envs
        if num_envs_global < self.env_offset + self.num_envs:
            raise ValueError(f"num_envs_global {num_envs_global} < env_offset + num_envs "
                             f"{self.env_offset + self.num_envs}")
        self.num_envs_global = int(num_envs_global)

        # ---- asset + terrain + derived params (legged_robot.py:1162-1319, 1417-1429) ----
        asset_file = cfg.asset.file.format(MINI_GYM_ROOT_DIR=MINI_GYM_ROOT_DIR)
        self.robot = load_robot(asset_file)
        self.num_bodies = self.robot["num_bodies"]
        self.num_dof = self.num_dofs = 12
        self.dof_names = self.robot["dof_names"]
        self.body_names = self.robot["body_names"]
        self.custom_origins = cfg.terrain.mesh_type in ("heightfield", "trimesh")
        self.terrain = None
        terrain_mesh = 0
        if self.custom_origins:
            terrain_mesh = self._create_terrain()
        self._P = lparams.build_params(cfg, self.robot, auto_reset=not self.legacy_fork,
                                       solver_iterations=solver_iterations, terrain_mesh=terrain_mesh)
        if eval_cfg is not None:
            # one kernel parameter block serves both groups: the eval cfg may differ from the train cfg only in
            # what the host applies per group (command ranges / curriculum, reset logging)
            Pe = lparams.build_params(eval_cfg, self.robot, auto_reset=not self.legacy_fork,
                                      solver_iterations=solver_iterations, terrain_mesh=terrain_mesh)
            # the eval tiles' teleport x offset is the one per-group kernel parameter
            self._P.num_train_envs = self.num_train_envs
            self._P.teleport_x_offset_eval = Pe.teleport_x_offset
            Pe.teleport_x_offset, Pe.teleport_x_offset_eval = self._P.teleport_x_offset, Pe.teleport_x_offset
            Pe.num_train_envs = self._P.num_train_envs
            def differs(f):
                a, b = getattr(self._P, f), getattr(Pe, f)
                return bytes(a) != bytes(b) if isinstance(a, C.Array) else a != b
            diff = [f for f, _ in type(self._P)._fields_ if differs(f)]
            if diff:
                raise NotImplementedError(f"eval_cfg differs from cfg in per-step kernel parameters {diff}; "
                                          "only host-side (command / curriculum) differences are supported")
        self._M = lparams.build_model(self.robot)
        self.sim_params = Section(dt=lparams.sim_dt(cfg))
        self.dt = cfg.control.decimation * self.sim_params.dt
        self.max_episode_length = cfg.env.max_episode_length
        self.obs_scales = cfg.normalization.obs_scales
        self.reward_scales = {k: v for k, v in lparams.reward_layout(cfg)[1].items()}
        self.reward_names = [k for k in self.reward_scales if k != "termination"]
        feet, pen, term = lparams.body_sets(cfg, self.robot)
        self.feet_indices = torch.tensor(feet, dtype=torch.long, device=self.device)
        self.penalised_contact_indices = torch.tensor(pen, dtype=torch.long, device=self.device)
        self.termination_contact_indices = torch.tensor(term, dtype=torch.long, device=self.device)

        # ---- sim ----
        L = _abi.lib()
        self._L = L
        self._sim = C.c_void_p()
        torch.cuda.set_device(self.device)
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        _abi.check(L.lrl_sim_create(C.byref(self._M), C.byref(self._P), C.c_int32(self.num_envs),
                                    C.c_int64(env_offset), C.c_uint64(self.seed), C.c_int32(dev_index),
                                    C.byref(self._sim)))
        self._dev_index = dev_index
        if terrain_mesh:  # gym.add_triangle_mesh / add_heightfield (legged_robot.py:1122-1160)
            t = self.terrain
            if cfg.terrain.mesh_type == "trimesh":
                vtx = t.vertices
            else:  # PhysX height field: the unmoved grid
                vtx, _ = convert_heightfield_to_trimesh(t.height_field_raw, cfg.terrain.horizontal_scale,
                                                        cfg.terrain.vertical_scale, None)
            vtx = np.ascontiguousarray(vtx, np.float32)
            hs = np.ascontiguousarray(t.heightsamples, np.int16)
            _abi.check(L.lrl_sim_set_terrain(self._sim, vtx.ctypes.data_as(C.c_void_p), hs.ctypes.data_as(C.c_void_p),
                                             C.c_int32(hs.shape[0]), C.c_int32(hs.shape[1])))
        self.height_samples = (torch.tensor(self.terrain.heightsamples).to(self.device)
                               if self.terrain is not None else None)
        T = self._tensor
        self.root_states = self.all_root_states = T(_abi.T_ROOT_STATE)
        self.dof_pos = T(_abi.T_DOF_POS)
        self.dof_vel = T(_abi.T_DOF_VEL)
        self.contact_forces = T(_abi.T_CONTACT_FORCE)
        self.rigid_body_state = T(_abi.T_RIGID_BODY_STATE)
        self.torques = T(_abi.T_TORQUES)
        self.actions = T(_abi.T_ACTIONS)
        self.last_actions = T(_abi.T_LAST_ACTIONS)
        self.last_dof_vel = T(_abi.T_LAST_DOF_VEL)
        self.last_root_vel = T(_abi.T_LAST_ROOT_VEL)
        self.commands = T(_abi.T_COMMANDS)
        self.obs_buf = T(_abi.T_OBS)
        self.privileged_obs_buf = T(_abi.T_PRIV_OBS)
        self.obs_history_buf = T(_abi.T_OBS_HISTORY)
        self.rew_buf = T(_abi.T_REWARD)
        self._reset_u8 = T(_abi.T_RESET)
        self._time_out_u8 = T(_abi.T_TIME_OUT)
        self.episode_length_buf = T(_abi.T_EPISODE_LENGTH)
        self._episode_sums = T(_abi.T_EPISODE_SUMS)
        self._command_sums = T(_abi.T_COMMAND_SUMS)
        self.feet_air_time = T(_abi.T_FEET_AIR_TIME)
        self._last_contacts_u8 = T(_abi.T_LAST_CONTACTS)
        self.friction_coeffs = T(_abi.T_FRICTION)
        self.restitutions = T(_abi.T_RESTITUTION)
        self.payloads = T(_abi.T_PAYLOAD)
        self.com_displacements = T(_abi.T_COM_DISPLACEMENT)
        self.motor_strengths = T(_abi.T_MOTOR_STRENGTH)
        self.Kp_factors = T(_abi.T_KP_FACTOR)
        self.Kd_factors = T(_abi.T_KD_FACTOR)
        self.env_origins = T(_abi.T_ENV_ORIGINS)
        self.base_lin_vel = T(_abi.T_BASE_LIN_VEL)
        self.base_ang_vel = T(_abi.T_BASE_ANG_VEL)
        self.projected_gravity = T(_abi.T_PROJECTED_GRAVITY)
        self.joint_pos_target = T(_abi.T_JOINT_POS_TARGET)
        self.base_quat = self.root_states[:, 3:7]
        keys = list(self.reward_scales)
        self.episode_sums = {k: self._episode_sums[i] for i, k in enumerate(keys + ["total"])}
        # eval-env episode results (legged_robot.py:1101-1105): -1 = not finished in this evaluation batch
        self.episode_sums_eval = {k: -torch.ones(self.num_envs, device=self.device) for k in keys}
        self.episode_sums_eval["total"] = torch.zeros(self.num_envs, device=self.device)
        self.command_sums = {k: self._command_sums[i] for i, k in enumerate(
            keys + ["lin_vel_raw", "ang_vel_raw", "lin_vel_residual", "ang_vel_residual", "ep_timesteps"])}
        self.default_dof_pos = torch.tensor(self._P.default_dof_pos[:], device=self.device).unsqueeze(0)
        self.p_gains = torch.tensor(self._P.p_gains[:], device=self.device)
        self.d_gains = torch.tensor(self._P.d_gains[:], device=self.device)
        self.torque_limits = torch.tensor(self._P.torque_limits[:], device=self.device)
        self.dof_pos_limits = torch.stack([torch.tensor(self._P.soft_dof_pos_lower[:]),
                                           torch.tensor(self._P.soft_dof_pos_upper[:])], 1).to(self.device)
        self.base_init_state = torch.tensor(self._P.base_init_state[:], device=self.device)
        self.default_body_mass = self.robot["base_mass"]
        # _get_heights runs inside the step kernel (legged_robot.py:584-585); 0 without a scan (:979)
        self.measured_heights = T(_abi.T_MEASURED_HEIGHTS) if cfg.terrain.measure_heights else 0
        if cfg.terrain.measure_heights:
            self.height_points = torch.zeros(self.num_envs, len(lparams.height_points(cfg)), 3, device=self.device)
            self.height_points[:, :, :2] = torch.tensor(lparams.height_points(cfg), device=self.device)
        self.common_step_counter = 0
        self.extras = _LazyExtras(self)
        self.record_now = False
        self.complete_video_frames = []

        # ---- origins, DR draws at creation (legged_robot.py:1216-1231, 1385-1415, 519-542) ----
        self._set_env_origins()
        self.all_root_states[:, 0:3] = self.env_origins
        self.all_root_states[:, 3:7] = torch.tensor([0.0, 0.0, 0.0, 1.0], device=self.device)
        self.all_root_states[:, 7:13] = 0.0
        dr = cfg.domain_rand
        which = (int(dr.randomize_base_mass) | (int(dr.randomize_com_displacement) << 1) |
                 (int(dr.randomize_friction) << 2) | (int(dr.randomize_restitution) << 3))
        arr = lambda r: (C.c_float * 2)(*[float(x) for x in r])
        _abi.check(L.lrl_sim_randomize(self._sim, arr(dr.friction_range), arr(dr.restitution_range),
                                       arr(dr.added_mass_range), arr(dr.com_displacement_range), C.c_uint32(which),
                                       self._stream()))
        if initial_dynamics_dict is not None:
            for k, v in initial_dynamics_dict.items():
                if hasattr(self, k) and isinstance(getattr(self, k), torch.Tensor):
                    getattr(self, k).copy_(v.to(self.device).view_as(getattr(self, k)))
        self._init_command_distribution()
        self.env_command_bins_t = torch.zeros(self.num_envs, device=self.device)
        self._ids_all = torch.arange(self.num_envs, dtype=torch.int32, device=self.device)
        self._due_next = None  # (episode_length_buf version, env ids due for command resampling next step)
        self._step_timer = None  # optional section timer of step() (scripts/step_timing.py)
        # pinned staging of the upstream-reset path's host->device data (ids, resampled commands, command bins)
        self._up = _Upload(self.device, 64 * self.num_envs + 4096) if str(self.device).startswith("cuda") else None
        self._sums_host = None  # (command_sums version, host copy of the two tracking rows) between a step's sync
        keys = list(self.reward_scales)  # and the resampling it feeds
        self._track_rows = [keys.index("tracking_lin_vel"), keys.index("tracking_ang_vel")] \
            if "tracking_lin_vel" in keys and "tracking_ang_vel" in keys else None
        # the upstream step without a host round trip (legacy_fork=False, one process, no eval group): reset ids,
        # command curriculum (lrl_sim_curriculum_resample_dev), terrain curriculum, episode logging, reset and
        # observation launches all read device-side lists and counts (_step_device).  LRL_DEVICE_RESETS=0 or
        # device_resets=False keeps the host path (one device->host copy per step), the check for this one.
        if device_resets is None:
            # (default on: 2.81-2.82 M against 2.59-2.63 M env-steps/s on configs[2], profiles/r4u_sec_ab.jsonl)
            device_resets = os.environ.get("LRL_DEVICE_RESETS", "1") != "0"
        self._dev_path = bool(device_resets) and not self.legacy_fork and self._dist is None and eval_cfg is None \
            and self._track_rows is not None and len(self._curriculum.keys) == 3
        self._dcur = None      # device curriculum buffers (allocated at the first device step)
        self._dev_auth = False  # True: the device copy of the curriculum / env bins is the current one
        self.init_done = True

    # ------------------------------------------------------------- command curriculum state (host mirror of the device)
    @property
    def curriculum(self):
        """RewardThresholdCurriculum (legged_robot.py:1056-1072).  On the device-reset path the device holds the current
        state; reading this refreshes the host object from it (and hands the state back to the host until the next
        step uploads it again)."""
        self._dev_sync_down()
        return self._curriculum

    @curriculum.setter
    def curriculum(self, c):
        self._curriculum = c
        self._dev_auth = False

    @property
    def env_command_bins(self):
        self._dev_sync_down()
        return self._env_command_bins

    @env_command_bins.setter
    def env_command_bins(self, b):
        self._env_command_bins = b
        self._dev_auth = False

    def _dev_sync_down(self):
        if not getattr(self, "_dev_auth", False):
            return
        d, cur = self._dcur, self._curriculum
        st = d["state"].cpu().numpy()
        if st[2]:
            raise ValueError({1: "probabilities contain NaN", 2: "probabilities are not non-negative"}.get(
                int(st[2]), "probabilities do not sum to 1"))
        cur.weights[:] = d["weights"].cpu().numpy()
        cur.episode_reward_lin[:] = d["ep_rew_lin"].cpu().numpy()
        cur.episode_reward_ang[:] = d["ep_rew_ang"].cpu().numpy()
        cur._mt_key[:] = d["mt_key"].cpu().numpy().view(np.uint32)
        cur._mt_pos[0] = int(st[1])
        cur._rng_obj = None
        self._env_command_bins[:] = d["env_bins"].cpu().numpy()
        self._dev_auth = False

    def _dev_upload(self):
        """The host curriculum / env bins into the device buffers (first device step, or after host-side access)."""
        cur, dev = self._curriculum, self.device
        cur._sync_from_rng()
        if self._dcur is None:
            n = self.num_envs
            axes = np.concatenate([cur.cfg[k] for k in cur.keys]).astype(np.float64)
            d = dict(weights=torch.zeros(len(cur), dtype=torch.float64, device=dev),
                     cdf=torch.zeros(len(cur), dtype=torch.float64, device=dev),
                     state=torch.zeros(4, dtype=torch.int32, device=dev),
                     mt_key=torch.zeros(624, dtype=torch.int32, device=dev),
                     ep_rew_lin=torch.zeros(len(cur), dtype=torch.float64, device=dev),
                     ep_rew_ang=torch.zeros(len(cur), dtype=torch.float64, device=dev),
                     env_bins=torch.zeros(n, dtype=torch.int64, device=dev),
                     env_bins_f=torch.zeros(n, dtype=torch.float32, device=dev),
                     command_area=torch.zeros(1, dtype=torch.float64, device=dev),
                     axes=torch.from_numpy(axes).to(dev),
                     words=torch.zeros(8 * n, dtype=torch.int32, device=dev),
                     draws=torch.zeros(4 * n, dtype=torch.float64, device=dev),
                     ids=[torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)],
                     cnt=torch.zeros(2, dtype=torch.int32, device=dev),
                     means=torch.full((self._episode_sums.shape[0],), float("nan"), device=dev),
                     level_mean=torch.zeros((), device=dev))
            desc = _abi.LrlDevCurriculum()
            for k in ("weights", "cdf", "state", "mt_key", "ep_rew_lin", "ep_rew_ang", "env_bins", "env_bins_f",
                      "command_area", "axes", "words", "draws"):
                setattr(desc, k, d[k].data_ptr())
            desc.half[:] = [float(cur.bin_sizes[k]) / 2 for k in cur.keys]
            desc.nx, desc.ny, desc.nz = (cur.ls[k] for k in cur.keys)
            d["desc"] = desc
            self._dcur = d
        d = self._dcur
        d["weights"].copy_(torch.from_numpy(np.ascontiguousarray(cur.weights, np.float64)))
        d["ep_rew_lin"].copy_(torch.from_numpy(np.ascontiguousarray(cur.episode_reward_lin, np.float64)))
        d["ep_rew_ang"].copy_(torch.from_numpy(np.ascontiguousarray(cur.episode_reward_ang, np.float64)))
        d["mt_key"].copy_(torch.from_numpy(cur._mt_key.view(np.int32).copy()))
        d["state"].copy_(torch.tensor([0, int(cur._mt_pos[0]), 0, 0], dtype=torch.int32))
        bins = np.ascontiguousarray(self._env_command_bins, np.int64)
        d["env_bins"].copy_(torch.from_numpy(bins))
        if self.env_command_bins_t is not d["env_bins_f"]:  # (the bins the last reset exposed, not the current ones)
            d["env_bins_f"].copy_(self.env_command_bins_t.reshape(-1)[:self.num_envs].to(torch.float32))
        self._dev_auth = True

    # -------------------------------------------------------------------------------- plumbing
    def _tensor(self, tid):
        d = _abi.LrlTensor()
        _abi.check(self._L.lrl_sim_tensor(self._sim, C.c_int32(tid), C.byref(d)))
        return _dlpack.wrap(d, self._dev_index)

    def _stream(self):
        return _abi.stream_of(self.device)

    def close(self):
        if getattr(self, "_sim", None):
            torch.cuda.synchronize(self.device)
            self._L.lrl_sim_destroy(self._sim)
            self._sim = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def reset_buf(self):
        return self._reset_u8.view(torch.bool)

    @property
    def time_out_buf(self):
        return self._time_out_u8.bool()

    @property
    def last_contacts(self):
        return self._last_contacts_u8.bool()

    # -------------------------------------------------------------------------------- terrain
    def _create_terrain(self):
        """create_sim's terrain (legged_robot.py:426-441): the Terrain tiles of the train cfg (and the eval cfg's
        tiles below them), generated with numpy's global RNG seeded by the env seed so every rank builds the
        same map.  Returns 1 when the ground is a mesh (some height is non-zero), 0 when it is the plane z = 0
        (the Mini Cheetah preset's all-flat trimesh), which keeps the plane contact path."""
        et = self.eval_cfg.terrain if self.eval_cfg is not None else None
        state = np.random.get_state()
        np.random.seed(self.seed)
        try:
            self.terrain = Terrain(self.cfg.terrain, self.num_train_envs, et, self.num_eval_envs)
        finally:
            np.random.set_state(state)
        return int(np.any(self.terrain.height_field_raw != 0))

    def _groups(self, env_ids=None):
        """_call_train_eval (legged_robot.py:456-469): (ids, cfg) of the train and eval envs among env_ids."""
        ids = torch.arange(self.num_envs, device=self.device) if env_ids is None else env_ids
        if self.eval_cfg is None:
            return [(ids, self.cfg)] if len(ids) else []
        out = [(ids[ids < self.num_train_envs], self.cfg)]
        if self.eval_cfg is not None:
            out.append((ids[ids >= self.num_train_envs], self.eval_cfg))
        return [(i, c) for i, c in out if len(i)]

    def _set_env_origins(self):
        """_get_env_origins (legged_robot.py:1385-1415), per train / eval group"""
        cfg, n = self.cfg, self.num_envs
        if self.custom_origins:
            g = torch.Generator().manual_seed(self.seed)
            self.terrain_levels = torch.zeros(n, dtype=torch.long, device=self.device)
            self.terrain_types = torch.zeros(n, dtype=torch.long, device=self.device)
            for ids, c in self._groups():
                t = c.terrain
                max_l = t.num_rows - 1 if not t.curriculum else t.max_init_terrain_level
                min_l = 0 if not t.curriculum else t.min_init_terrain_level
                if not 0 <= min_l <= max_l < t.num_rows:  # the reference would index terrain_origins out of range
                    raise IndexError(f"initial terrain levels [{min_l}, {max_l}] outside the {t.num_rows} terrain rows "
                                     "(Cfg.terrain.max_init_terrain_level)")
                k = len(ids)
                # the train group of a shard draws over the global train envs and keeps its slice (the eval group is
                # per process)
                lo, kg = (self.env_offset, self.num_envs_global - (self.num_envs - self.num_train_envs)) \
                    if c is self.cfg else (0, k)
                lv = torch.randint(min_l, max_l + 1, (kg,), generator=g)[lo:lo + k]
                ty = torch.div(torch.arange(kg), (kg / t.num_cols), rounding_mode="floor").long()[lo:lo + k]
                self.terrain_levels[ids] = lv.to(self.device)
                self.terrain_types[ids] = ty.to(self.device)
                t.max_terrain_level = t.num_rows
                t.terrain_origins = torch.from_numpy(t.env_origins).to(self.device).float()
                self.env_origins[ids] = t.terrain_origins[self.terrain_levels[ids], self.terrain_types[ids]]
            self._level_gen = torch.Generator(device=self.device).manual_seed(self.seed + 1)
        else:  # the global grid of all ranks' envs, this shard's slice
            ng, lo = self.num_envs_global, self.env_offset
            num_cols = np.floor(np.sqrt(ng))
            num_rows = np.ceil(ng / num_cols)
            xx, yy = torch.meshgrid(torch.arange(num_rows), torch.arange(num_cols), indexing="ij")
            sp = cfg.env.env_spacing
            self.env_origins[:, 0] = (sp * xx.flatten()[lo:lo + n]).to(self.device)
            self.env_origins[:, 1] = (sp * yy.flatten()[lo:lo + n]).to(self.device)
            self.env_origins[:, 2] = 0.0

    # -------------------------------------------------------------------------------- commands
    def _init_command_distribution(self):
        """legged_robot.py:1056-1072"""
        c = self.cfg.commands
        self._curriculum = RewardThresholdCurriculum(
            seed=c.curriculum_seed, x_vel=(c.limit_vel_x[0], c.limit_vel_x[1], 51),
            y_vel=(c.limit_vel_y[0], c.limit_vel_y[1], 2), yaw_vel=(c.limit_vel_yaw[0], c.limit_vel_yaw[1], 51))
        self._env_command_bins = np.zeros(self.num_envs, dtype=int)
        low = np.array([c.lin_vel_x[0], c.lin_vel_y[0], c.ang_vel_yaw[0]])
        high = np.array([c.lin_vel_x[1], c.lin_vel_y[1], c.ang_vel_yaw[1]])
        self._curriculum.set_to(low=low, high=high)
        self._dev_auth = False

    def _dist_count(self, k):
        """Sum over ranks of a local count (one small all-reduce)."""
        dist = self._dist
        dev = self.device if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([k], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        return int(t.item())

    def _dist_gather_rows(self, rows):
        """All ranks' rows (float64 [k, m]) concatenated in rank order, and this rank's first row in it."""
        dist = self._dist
        dev = self.device if dist.get_backend() == "nccl" else "cpu"
        world, rank = dist.get_world_size(), dist.get_rank()
        cnt = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
        cnts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(cnts, cnt)
        cnts = [int(c.item()) for c in cnts]
        kmax = max(cnts)
        if kmax == 0:
            return rows[:0], 0
        buf = torch.zeros(kmax, rows.shape[1], dtype=torch.float64, device=dev)
        buf[:rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows, np.float64)).to(dev)
        bufs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(bufs, buf)
        return np.concatenate([b[:c].cpu().numpy() for b, c in zip(bufs, cnts)]), sum(cnts[:rank])

    def resample_commands(self, env_ids, _ids_host=None, _ids32=None, _bins_to=None):
        """_resample_commands (legged_robot.py:595-626); disconnected in the fork (Q3), callable here.
        ``_ids_host``: the same ids as a numpy array when the caller already has them on the host; ``_ids32``: as a
        device int32 array; ``_bins_to``: a device float tensor that receives all envs' command bins (reset_idx's
        env_bins) in the same launch."""
        if env_ids is not None and len(env_ids) == 0 and self._dist is None:  # (ranks join the collective update
            return  # with no envs of their own)
        if _ids_host is not None and len(_ids_host) == 0 and self._dist is None:
            return
        # env_ids None: the ids exist only on the host (_ids_host) and travel with the commands' upload
        ids = None if (env_ids is None or _ids32 is not None) else torch.as_tensor(env_ids, device=self.device,
                                                                                   dtype=torch.long)
        timesteps = int(self.cfg.commands.resampling_time / self.dt)
        ep_len = min(self.cfg.env.max_episode_length, timesteps)
        # both tracking sums in one device->host copy (float32 division on the device, as torch does)
        ids_np = (ids if ids is not None else _ids32).cpu().numpy() if _ids_host is None else _ids_host
        hs = self._sums_host
        if hs is not None and _ids_host is not None and hs[0] == self._command_sums._version:
            # the step's device->host copy (float32 sums / ep_len in float32, as torch divides on the device)
            lin, ang = hs[1][:, ids_np] / np.float32(ep_len)
            hs[1][:, ids_np] = 0.0  # mirrors the zeroing below
        else:
            ids_d = ids if ids is not None else torch.as_tensor(ids_np, device=self.device, dtype=torch.long)
            lin, ang = (self._command_sums[self._track_rows][:, ids_d] / ep_len).cpu().numpy()
        lin_thr = self.cfg.commands.forward_curriculum_threshold * self.reward_scales["tracking_lin_vel"]
        ang_thr = self.cfg.commands.yaw_curriculum_threshold * self.reward_scales["tracking_ang_vel"]
        old_bins = self.env_command_bins[ids_np]
        if self._dist is None:
            self.curriculum.update(old_bins, lin, ang, lin_thr, ang_thr, local_range=0.5)
            new_cmds, new_bins = self.curriculum.sample(batch_size=len(ids_np))
        else:  # the same update / draw on every rank over all ranks' envs, then this rank's rows
            rows, off = self._dist_gather_rows(np.stack([old_bins.astype(np.float64), np.asarray(lin, np.float64),
                                                         np.asarray(ang, np.float64)], 1))
            if len(rows) == 0:
                return
            self.curriculum.update(rows[:, 0].astype(old_bins.dtype), rows[:, 1].astype(np.float32),
                                   rows[:, 2].astype(np.float32), lin_thr, ang_thr, local_range=0.5)
            new_cmds, new_bins = self.curriculum.sample(batch_size=len(rows))
            new_cmds, new_bins = new_cmds[off:off + len(ids_np)], new_bins[off:off + len(ids_np)]
        self.env_command_bins[ids_np] = new_bins
        # commands[:, :3] = float32(cmds); commands[:, :2] *= (norm(commands[:, :2]) > 0.2): float32 on the host
        c = new_cmds.astype(np.float32)
        keep = (np.sqrt(c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]) > np.float32(0.2)).astype(np.float32)
        c[:, 0] *= keep
        c[:, 1] *= keep
        # one pinned upload (int32 ids unless the caller has them on the device, the commands, the bins when asked for)
        # and one launch: commands[ids, :3] = c, command_sums[:, ids] = 0, bins (lrl_sim_apply_commands)
        arrays = ([] if _ids32 is not None else [np.asarray(ids_np, np.int32)]) + [c]
        if _bins_to is not None:
            arrays.append(self.env_command_bins.astype(np.float32))
        up = self._up.put(*arrays)
        ids32 = _ids32 if _ids32 is not None else up[0]
        cd = up[0 if _ids32 is not None else 1]
        bins = up[-1] if _bins_to is not None else None
        _abi.check(self._L.lrl_sim_apply_commands(
            self._sim, C.c_void_p(ids32.data_ptr()), C.c_int32(len(ids_np)), C.c_void_p(cd.data_ptr()),
            C.c_void_p(bins.data_ptr() if bins is not None else 0),
            C.c_void_p(_bins_to.data_ptr() if _bins_to is not None else 0),
            C.c_int32(len(_bins_to) if _bins_to is not None else 0), self._stream()))
        # (the kernel's writes do not move the tensors' version counters: the step's host copy of the tracking sums,
        # zeroed above for these ids, stays valid)

    # -------------------------------------------------------------------------------- API
    def step(self, actions, _history=False):
        """VelocityTrackingEasyEnv.step: returns (obs, rew, done, extras)."""
        if actions.device != self.device or actions.dtype != torch.float32 or not actions.is_contiguous():
            actions = actions.to(self.device, torch.float32).contiguous()
        if actions.shape != (self.num_envs, self.num_actions):
            raise ValueError(f"actions must be [{self.num_envs}, {self.num_actions}], got {tuple(actions.shape)}")
        flags = _abi.STEP_PHYSICS | (_abi.STEP_HISTORY if _history else 0)
        if self._dev_path:
            return self._step_device(actions, flags)
        tm = self._step_timer  # scripts/step_timing.py: host time per section of this method (None: off)
        if tm is not None:
            tm.mark("entry")
        if not self.legacy_fork:  # _post_physics_step_callback resampling (legged_robot.py:578-581): the
            # envs whose episode length reaches a multiple of resampling_time in this step, before its rewards
            interval = self._resample_interval()
            cached = self._due_next
            if cached is not None and cached[0] == self.episode_length_buf._version:
                due, due_np = None, cached[1]  # known from the previous step's single device->host copy (the ids
                # reach the device with the resampled commands' upload)
            else:  # first step, or episode_length_buf written by a caller since: host ids from the fresh set
                due = ((self.episode_length_buf + 1) % interval == 0).nonzero(as_tuple=False).flatten()
                due_np = due.cpu().numpy()
            # (with several ranks every rank takes part whenever any rank has envs to resample)
            if (len(due_np) > 0) if self._dist is None else (self._dist_count(len(due_np)) > 0):
                self.resample_commands(due, due_np)
        self._sums_host = None  # the kernel below changes the command sums
        if tm is not None:
            tm.mark("pre_resample")
        _abi.check(self._L.lrl_sim_step(self._sim, C.c_void_p(actions.data_ptr()), C.c_uint32(flags), self._stream()))
        self.common_step_counter += 1
        if not self.legacy_fork:  # reset_idx of the terminated / timed-out envs, then their observations
            # one device->host copy per step: bit 0 = reset now, bit 1 = due for resampling next step (episode
            # length after this step's resets: 0 for the reset envs)
            # length after this step's resets: 0 for the reset envs), rows 1-2 = the tracking command sums the
            # curriculum update of the envs resampled next (resets now, due ones before the next kernel) reads
            eplen = self.episode_length_buf
            # (lrl_sim_step_code: the code and the two tracking rows computed on the device and copied into a pinned
            # host buffer in one call — the torch form was eight small ops and a pageable copy)
            tr = self._track_rows if self._track_rows is not None else (-1, -1)
            if getattr(self, "_code_host", None) is None:
                self._code_host = torch.empty(3 * self.num_envs, dtype=torch.float32, pin_memory=True).numpy()
                self._rid32 = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
            # (the reset ids are compacted on the device in the same call: no host -> device upload of them)
            _abi.check(self._L.lrl_sim_step_code(self._sim, C.c_int32(interval), C.c_int32(tr[0]), C.c_int32(tr[1]),
                                                 C.c_void_p(self._code_host.ctypes.data),
                                                 C.c_void_p(self._rid32.data_ptr()), self._stream()))
            pack = self._code_host.reshape(3, self.num_envs)
            code = pack[0].astype(np.uint8)
            if self._track_rows is not None:
                self._sums_host = (self._command_sums._version, pack[1:3])
            if tm is not None:
                tm.mark("launch_and_sync")
            rst = code & 1
            ids_np = np.flatnonzero(rst)
            due_np = np.flatnonzero((code >> 1) & ((rst == 0) | (interval == 1)))
            if (len(ids_np) > 0) if self._dist is None else (self._dist_count(len(ids_np)) > 0):
                ids32 = self._rid32[:len(ids_np)]  # lrl_sim_step_code's compaction (ascending, as ids_np)
                if tm is not None:
                    tm.mark("ids_h2d")
                self.reset_idx(ids32, ids_np, _ids32=ids32)
                _abi.check(self._L.lrl_sim_observe_idx(self._sim, C.c_void_p(ids32.data_ptr()), C.c_int32(len(ids32)),
                                                       C.c_uint32(flags), self._stream()))
            self._due_next = (eplen._version, due_np)
            if tm is not None:
                tm.mark("reset_idx_observe")
        ex = self.extras
        ex["privileged_obs"] = self.privileged_obs_buf
        ex["joint_vel_target"] = torch.zeros(12)
        self._register_extras(ex)
        if tm is not None:
            tm.mark("extras")
        return self.obs_buf, self.rew_buf, self._reset_u8.view(torch.bool), self.extras

    # rows of lrl_sim_extras_snapshot (include/lrl.h LRL_EXTRAS_*): key -> (first row, rows)
    _EXTRAS_ROWS = 77
    _EXTRAS = {"joint_pos": (0, 12), "joint_vel": (12, 12), "joint_pos_target": (24, 12), "body_linear_vel": (36, 3),
               "body_angular_vel": (39, 3), "body_linear_vel_cmd": (42, 2), "body_angular_vel_cmd": (44, 2),
               "contact_states": (46, 4), "foot_positions": (50, 12), "body_pos": (62, 3), "torques": (65, 12)}

    def _register_extras(self, ex):
        """The step's numpy extras as lazy reads of one device snapshot taken now (see _LazyExtras).
        (LRL_EXTRAS_SNAPSHOT=0, a development switch for A/B timing: lazy reads of the live tensors instead.)"""
        n = self.num_envs
        if not _SNAPSHOT_EXTRAS:
            live = {"joint_pos": lambda: self.dof_pos, "joint_vel": lambda: self.dof_vel,
                    "joint_pos_target": lambda: self.joint_pos_target, "body_linear_vel": lambda: self.base_lin_vel,
                    "body_angular_vel": lambda: self.base_ang_vel, "body_linear_vel_cmd": lambda: self.commands[:, 0:2],
                    "body_angular_vel_cmd": lambda: self.commands[:, 2:],
                    "contact_states": lambda: self.contact_forces[:, self.feet_indices, 2] > 1.0,
                    "foot_positions": self._foot_positions, "body_pos": lambda: self.root_states[:, 0:3],
                    "torques": lambda: self.torques}
            for key, fn in live.items():
                ex.set_lazy(key, lambda fn=fn: fn().cpu().numpy().copy())
            return
        snap = torch.empty(self._EXTRAS_ROWS, n, device=self.device)
        _abi.check(self._L.lrl_sim_extras_snapshot(self._sim, C.c_void_p(snap.data_ptr()), self._stream()))
        nf = len(self.feet_indices)

        def read(key):
            r0, k = self._EXTRAS[key]
            if key == "contact_states":
                return (snap[r0:r0 + nf].t() > 0.5).cpu().numpy().copy()
            if key == "foot_positions":
                return snap[r0:r0 + 3 * nf].t().reshape(n, nf, 3).cpu().numpy().copy()
            return snap[r0:r0 + k].t().cpu().numpy().copy()
        for key in self._EXTRAS:
            ex.set_lazy(key, lambda key=key: read(key))

    _INT32_MAX = 2 ** 31 - 1

    def _resample_interval(self):
        """resampling_time / dt in steps, clamped to int32 for the device launches: an interval past the int32 range
        (e.g. the reference's eval settings, resampling_time = 1e9) is never reached by an int32 episode length, so
        the clamp changes no decision."""
        return min(int(self.cfg.commands.resampling_time / self.dt), self._INT32_MAX)

    def _step_device(self, actions, flags):
        """step() on the upstream path with every reset / resampling decision on the device (no host wait): the same
        launches and draws as the host path below (legged_robot.py:139-188, 227-290, 578-581, 595-626), with id lists
        and counts that never leave the device."""
        L, sim, st = self._L, self._sim, self._stream()
        if not self._dev_auth:
            self._dev_upload()
        d = self._dcur
        n = self.num_envs
        vp = lambda t: C.c_void_p(t.data_ptr())
        interval = self._resample_interval()
        # (max_episode_length is a float, np.ceil's; an integral value either way, as the divisor of the tracking sums)
        ep_len = int(min(self.cfg.env.max_episode_length, interval))
        lin_thr = self.cfg.commands.forward_curriculum_threshold * self.reward_scales["tracking_lin_vel"]
        ang_thr = self.cfg.commands.yaw_curriculum_threshold * self.reward_scales["tracking_ang_vel"]
        due, rst = d["ids"]
        cnt = d["cnt"]
        due_n, rst_n = C.c_void_p(cnt.data_ptr()), C.c_void_p(cnt.data_ptr() + 4)
        r0, r1 = self._track_rows

        def resample(ids, count, log_area):
            _abi.check(L.lrl_sim_curriculum_resample_dev(sim, C.byref(d["desc"]), vp(ids), C.c_int32(n), count,
                                                         C.c_int32(ep_len), C.c_int32(r0), C.c_int32(r1),
                                                         C.c_double(lin_thr), C.c_double(ang_thr), C.c_double(0.5),
                                                         C.c_int32(1), C.c_int32(log_area), st))
        # _post_physics_step_callback's resampling of the envs whose episode reaches a multiple of resampling_time
        _abi.check(L.lrl_sim_env_lists(sim, C.c_int32(1), C.c_int32(interval), vp(due), due_n, st))
        resample(due, due_n, 0)
        _abi.check(L.lrl_sim_step(sim, vp(actions), C.c_uint32(flags), st))
        self.common_step_counter += 1
        # reset_idx of the terminated / timed-out envs (legged_robot.py:227-290), then their observations
        _abi.check(L.lrl_sim_env_lists(sim, C.c_int32(0), C.c_int32(interval), vp(rst), rst_n, st))
        cfg = self.cfg
        if self.custom_origins and cfg.terrain.curriculum:
            t = cfg.terrain
            to = t.terrain_origins
            _abi.check(L.lrl_sim_terrain_curriculum_dev(
                sim, vp(rst), C.c_int32(n), rst_n, vp(self.terrain_levels), vp(self.terrain_types), vp(to),
                C.c_int32(to.shape[0]), C.c_int32(to.shape[1]), C.c_float(t.env_length / 2),
                C.c_float(cfg.env.episode_length_s), C.c_int32(t.max_terrain_level), st))
        c = cfg.commands
        if (c.command_curriculum or c.yaw_command_curriculum) and self.common_step_counter % cfg.env.max_episode_length == 0:
            k = int(cnt[1].item())  # (the uniform command-range curriculum's step: once per episode length, host sync)
            if k:
                self.update_command_curriculum(rst[:k].long(), cfg)
        # This step's logged values land in fresh buffers (an empty reset batch copies the previous step's), so the
        # dict published below holds values no later step overwrites, as the reference's fresh tensors per reset batch.
        ex = self.extras
        ep_host = dict.get(ex, "train/episode")
        if ep_host is not None and ep_host is not d.get("ep"):  # continue from what the host path logged last (reset())
            for i, k in enumerate(self.episode_sums):
                v = ep_host.get("rew_" + k)
                if isinstance(v, torch.Tensor) and v.numel() == 1:
                    d["means"][i].copy_(v.reshape(()))
            if "command_area" in ep_host:
                d["command_area"].fill_(float(ep_host["command_area"]))
            d["seen"] = True
        desc = d["desc"]
        bins_new = torch.empty_like(d["env_bins_f"])
        area_new = torch.empty_like(d["command_area"])
        desc.env_bins_f, desc.command_area = bins_new.data_ptr(), area_new.data_ptr()
        desc.env_bins_f_prev, desc.command_area_prev = d["env_bins_f"].data_ptr(), d["command_area"].data_ptr()
        resample(rst, rst_n, 1)
        desc.env_bins_f_prev = desc.command_area_prev = None
        d["env_bins_f"], d["command_area"] = bins_new, area_new
        es = self._episode_sums
        R = es.shape[0]
        pub = torch.empty(R + 1, device=self.device)  # [means of the last reset batch | terrain level]
        _abi.check(L.lrl_rows_mean_zero_dev(vp(es), C.c_int64(es.stride(0)), C.c_int32(R), vp(rst), C.c_int32(n), rst_n,
                                            vp(pub), vp(d["means"]), C.c_int32(1), st))
        d["means"] = pub[:R]
        t = cfg.terrain
        _abi.check(L.lrl_sim_reset_idx_dev(sim, vp(rst), C.c_int32(n), rst_n, C.c_int32(self._root_mode()),
                                           C.c_float(float(t.x_init_range)),
                                           C.c_float(float(t.y_init_range) - float(t.x_init_range)),
                                           C.c_float(float(t.x_init_offset)), C.c_float(float(t.y_init_offset)), st))
        _abi.check(L.lrl_sim_observe_idx_dev(sim, vp(rst), C.c_int32(n), rst_n, C.c_uint32(flags), st))
        self._due_next = None
        self._sums_host = None
        ep = d["ep"] = {"rew_" + k: m for k, m in zip(self.episode_sums, pub[:R].unbind(0))}
        if cfg.terrain.curriculum and self.custom_origins:
            torch.mean(self.terrain_levels[:self.num_train_envs], dim=0, dtype=torch.float32, out=pub[R])  # (one kernel)
            ep["terrain_level"] = pub[R]
        if c.command_curriculum:
            self.env_command_bins_t = bins_new
            ex["env_bins"] = bins_new[:self.num_train_envs]
            ep["command_area"] = area_new[0]
        if c.yaw_command_curriculum:
            ep["max_command_yaw"] = cfg.command_ranges["ang_vel_yaw"][1]
        if d.get("seen"):
            ex["train/episode"] = ep
        else:  # no reset logged yet: the key appears once one has been (the means are NaN until then), as the
            # reference's extras gain it at the first reset batch; deciding that reads one device value, on access only
            def seen(ep=ep, m0=pub[0]):
                if bool(torch.isnan(m0).item()):
                    return False
                d["seen"] = True
                return True
            ex.set_conditional("train/episode", ep, seen)
        if cfg.env.send_timeouts:
            ex["time_outs"] = self.time_out_buf[:self.num_train_envs]
        ex["privileged_obs"] = self.privileged_obs_buf
        ex["joint_vel_target"] = torch.zeros(12)
        self._register_extras(ex)
        return self.obs_buf, self.rew_buf, self._reset_u8.view(torch.bool), self.extras

    def kernel_timing(self, start):
        """Env-kernel launch time, the one definition bench.py and the scripts use: HIP events around each
        env_step_kernel launch of lrl_sim_step on its own stream (lrl_sim_timing; the history-shift launch before it
        is outside).  start=True begins recording; start=False stops and returns (mean ms, total ms, launches)."""
        ms, n = C.c_double(0.0), C.c_int64(0)
        _abi.check(self._L.lrl_sim_timing(self._sim, C.c_int32(1 if start else 0), C.byref(ms), C.byref(n)))
        if start:
            return None
        return (ms.value / n.value if n.value else float("nan")), ms.value, n.value

    def self_contact_stats(self, start):
        """lrl_sim_self_contact_stats: start=True zeroes the device counters and starts counting; start=False stops and
        returns {env_substeps_in_self_contact, self_pairs_in_contact, env_substeps_over_cap, self_pairs_dropped}."""
        out = (C.c_uint64 * 4)()
        _abi.check(self._L.lrl_sim_self_contact_stats(self._sim, C.c_int32(1 if start else 0), out))
        if start:
            return None
        return dict(zip(("env_substeps_in_self_contact", "self_pairs_in_contact", "env_substeps_over_cap",
                         "self_pairs_dropped"), (int(x) for x in out)))

    def _foot_positions(self):
        self.refresh_rigid_body_state()
        return self.rigid_body_state[:, self.feet_indices, 0:3]

    def refresh_rigid_body_state(self):
        _abi.check(self._L.lrl_sim_refresh_rigid_body_state(self._sim, self._stream()))

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self, horizon=0):
        return self.privileged_obs_buf

    def render(self, mode="rgb_array"):
        """BaseTask.render (base_task.py:92-118) draws through the Isaac Gym viewer / camera sensors; rendering is out of
        scope here (no viewer), so asking for a frame is an error, not a blank image."""
        raise NotImplementedError("no viewer / camera rendering in this framework (DESIGN.md §8)")

    def reset(self):
        """VelocityTrackingEasyEnv.reset (:66-69): reset all, then one zero-action step."""
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        obs, _, _, _ = self.step(torch.zeros(self.num_envs, self.num_actions, device=self.device))
        return obs

    def reset_idx(self, env_ids, _ids_host=None, _ids32=None):
        """legged_robot.py:227-290; train and eval envs (env id >= num_train_envs) go through their own cfg
        for the command curriculum (_call_train_eval, :456-469) and their own episode logging.  (_ids_host / _ids32:
        the same ids on the host and as a device int32 array, from step's upload.)"""
        env_ids = torch.as_tensor(env_ids, device=self.device)
        if env_ids.dtype not in (torch.int64, torch.int32):  # (int32 ids — the step's compaction — index as they are)
            env_ids = env_ids.long()
        if len(env_ids) == 0 and self._dist is None:  # (ranks join the collective curriculum steps with no envs)
            return
        self._due_next = None  # episode lengths change: the next step re-derives its resampling set
        tm = self._step_timer
        n_tr = self.num_train_envs
        if self.num_eval_envs:
            tr, ev = env_ids[env_ids < n_tr], env_ids[env_ids >= n_tr]
        else:
            tr, ev = env_ids, env_ids[:0]
        one_group = self.eval_cfg is None
        if _ids32 is None or not one_group:
            _ids32 = None
        if self.custom_origins:
            for ids, c in self._groups(env_ids):
                self._update_terrain_curriculum(ids, c, _ids32)
        if len(tr) or self._dist is not None:
            self.update_command_curriculum(tr, self.cfg)
        if len(ev) or (self._dist is not None and self.num_eval_envs):
            self.update_command_curriculum(ev, self.eval_cfg)
        if tm is not None:
            tm.mark("r_terrain_cmdcurr")
        bins_done = False
        if not self.legacy_fork:  # upstream reset_idx resamples the reset envs' commands
            bins_to = None
            if self.cfg.commands.command_curriculum:  # the env bins travel with the commands (one upload, one launch)
                if self.env_command_bins_t.shape != (self.num_envs,):
                    self.env_command_bins_t = torch.zeros(self.num_envs, device=self.device)
                bins_to, bins_done = self.env_command_bins_t, True
            self.resample_commands(env_ids, _ids_host, _ids32=_ids32, _bins_to=bins_to)
        if tm is not None:
            tm.mark("r_resample")
        # episode logging before the per-env sums are zeroed (:261-276)
        if len(tr):
            ep = {}
            es = self._episode_sums
            if es.stride(1) == 1 and es.is_cuda:  # means and zeroing in one launch (lrl_rows_mean_zero)
                tr32 = _ids32 if _ids32 is not None else tr.to(torch.int32).contiguous()
                means = torch.empty(es.shape[0], device=self.device)
                _abi.check(self._L.lrl_rows_mean_zero(C.c_void_p(es.data_ptr()), C.c_int64(es.stride(0)),
                                                      C.c_int32(es.shape[0]), C.c_void_p(tr32.data_ptr()),
                                                      C.c_int32(len(tr32)), C.c_void_p(means.data_ptr()), C.c_int32(1),
                                                      self._stream()))
            else:
                means = es[:, tr].mean(dim=1)
                es[:, tr] = 0.0
            for k, m in zip(self.episode_sums, means.unbind(0)):  # (one call for all the 0-d views)
                ep["rew_" + k] = m
            self.extras["train/episode"] = ep
        if len(ev):
            self.extras["eval/episode"] = {}
            for i, k in enumerate(self.episode_sums):  # keep the first finished episode of each eval env
                unset = ev[self.episode_sums_eval[k][ev] == -1]
                self.episode_sums_eval[k][unset] = self.episode_sums[k][unset]
            self._episode_sums[:, ev] = 0.0
        if tm is not None:
            tm.mark("r_episode_log")
        self._reset_device(env_ids, _ids32)
        if tm is not None:
            tm.mark("r_reset_device")
        ep = self.extras.get("train/episode")
        if ep is None:
            ep = self.extras["train/episode"] = {}
        if self.cfg.terrain.curriculum:  # :278-280
            ep["terrain_level"] = torch.mean(self.terrain_levels[:self.num_train_envs].float())
        if self.cfg.commands.command_curriculum:  # (torch.tensor(env_command_bins, dtype=float), via the pinned slot)
            if bins_done:
                pass  # written by resample_commands' launch
            elif self._up is not None:
                if self.env_command_bins_t.shape != (self.num_envs,):
                    self.env_command_bins_t = torch.zeros(self.num_envs, device=self.device)
                self.env_command_bins_t.copy_(self._up.put(self.env_command_bins.astype(np.float32))[0])
            else:
                self.env_command_bins_t = torch.tensor(self.env_command_bins, dtype=torch.float, device=self.device)
            self.extras["env_bins"] = self.env_command_bins_t[:self.num_train_envs]
            ep["command_area"] = np.sum(self.curriculum.weights) / self.curriculum.weights.shape[0]
        if self.cfg.commands.yaw_command_curriculum:  # :283-286
            ep["max_command_yaw"] = self.cfg.command_ranges["ang_vel_yaw"][1]
            if self.eval_cfg is not None:
                ev_ep = self.extras.get("eval/episode")
                if ev_ep is None:
                    ev_ep = self.extras["eval/episode"] = {}
                ev_ep["max_command_yaw"] = self.eval_cfg.command_ranges["ang_vel_yaw"][1]
        if self.cfg.env.send_timeouts:
            self.extras["time_outs"] = self.time_out_buf[:self.num_train_envs]
        if tm is not None:
            tm.mark("r_extras")

    def _root_mode(self):
        """_reset_root_states (legged_robot.py:714-755) as a reset_kernel root mode (lrl.h): the plane path writes
        all_root_states (mode 1); with custom origins the fork writes an advanced-index copy and pushes the unchanged
        all_root_states, so the root is left as it is (mode 0); upstream semantics (legacy_fork=False)
        place it at the origin plus the U[x_init_range, y_init_range] draw and the init offsets (mode 2)."""
        if not self.custom_origins:
            return 1
        return 0 if self.legacy_fork else 2

    def _reset_device(self, env_ids, _ids32=None):
        """The device part of reset_idx, one launch per train / eval group (each with its cfg's init ranges):
        _randomize_dof_props, _reset_dofs, _reset_root_states and the buffer zeroing (:247-259).  A test may set
        ``reset_uniforms`` ([len(env_ids), 5] device f32: motor strength, Kp, Kd, x, y per env id) to replace the
        draws of the next reset."""
        inj, self.reset_uniforms = getattr(self, "reset_uniforms", None), None
        mode = self._root_mode()
        groups = self._groups(env_ids) if len(env_ids) else []
        for ids, c in groups:
            ids32 = _ids32 if (_ids32 is not None and len(groups) == 1) else ids.to(torch.int32).contiguous()
            flags = 0
            if inj is not None:
                rows = inj if len(ids) == len(env_ids) else inj[torch.isin(env_ids, ids)]
                rows = rows.to(self.device, torch.float32).contiguous()
                _abi.check(self._L.lrl_sim_inject_reset_uniforms(self._sim, C.c_void_p(rows.data_ptr())))
                flags = _abi.STEP_INJECT_UNIFORM
            t = c.terrain
            _abi.check(self._L.lrl_sim_reset_idx_ex(
                self._sim, C.c_void_p(ids32.data_ptr()), C.c_int32(len(ids32)), C.c_int32(mode),
                C.c_float(float(t.x_init_range)), C.c_float(float(t.y_init_range) - float(t.x_init_range)),
                C.c_float(float(t.x_init_offset)),
                C.c_float(float(t.y_init_offset)), C.c_uint32(flags), self._stream()))
            if inj is not None:
                torch.cuda.current_stream(self.device).synchronize()  # rows must outlive the launch

    # torch.randint_like(levels, high) of _update_terrain_curriculum: None = the curriculum kernel's own counter-RNG draw
    # (global env id, step counter), the same on the host and device reset paths; tests set a callable (like, high) ->
    # int64 draws to inject the reference's draws
    _rand_levels = None

    def _torch_rand_levels(self, like, high):
        """The draws of the host torch form (tensors without a sim): a seeded device generator."""
        return torch.randint(0, high, like.shape, generator=self._level_gen, device=self.device, dtype=torch.int64)

    def _update_terrain_curriculum(self, env_ids, cfg, _ids32=None):
        """legged_robot.py:793-818: robots that walked past half a tile move a level up, those that covered less
        than half of their commanded distance move down (not both); past the last level a random level."""
        if not cfg.terrain.curriculum or not getattr(self, "init_done", False):
            return
        t = cfg.terrain
        if getattr(self, "_sim", None) is not None:  # one launch instead of ~25 indexed torch ops per reset
            rnd = None
            if self._rand_levels is not None:  # injected draws (tests)
                rnd = self._rand_levels(env_ids, t.max_terrain_level).contiguous()
                if rnd.dtype != torch.int64 or rnd.device != self.device or rnd.numel() < len(env_ids):
                    raise TypeError(f"terrain level draws must be int64 on {self.device} with one per env id, got "
                                    f"{rnd.dtype} on {rnd.device} [{rnd.numel()}] for {len(env_ids)} ids")
            ids32 = _ids32 if _ids32 is not None else env_ids.to(torch.int32).contiguous()
            to = t.terrain_origins
            _abi.check(self._L.lrl_sim_terrain_curriculum(
                self._sim, C.c_void_p(ids32.data_ptr()), C.c_int32(len(ids32)), C.c_void_p(self.terrain_levels.data_ptr()),
                C.c_void_p(self.terrain_types.data_ptr()), C.c_void_p(rnd.data_ptr() if rnd is not None else 0),
                C.c_void_p(to.data_ptr()),
                C.c_int32(to.shape[0]), C.c_int32(to.shape[1]), C.c_float(t.env_length / 2),
                C.c_float(cfg.env.episode_length_s), C.c_int32(t.max_terrain_level), self._stream()))
            return
        distance = torch.norm(self.root_states[env_ids, :2] - self.env_origins[env_ids, :2], dim=1)
        move_up = distance > t.env_length / 2
        move_down = (distance < torch.norm(self.commands[env_ids, :2], dim=1) * cfg.env.episode_length_s * 0.5) * ~move_up
        self.terrain_levels[env_ids] += 1 * move_up - 1 * move_down
        lv = self.terrain_levels[env_ids]
        draw = self._rand_levels if self._rand_levels is not None else self._torch_rand_levels
        self.terrain_levels[env_ids] = torch.where(lv >= t.max_terrain_level, draw(lv, t.max_terrain_level),
                                                   torch.clip(lv, 0))
        self.env_origins[env_ids] = t.terrain_origins[self.terrain_levels[env_ids], self.terrain_types[env_ids]]

    def _ids_mean(self, values, env_ids):
        """torch.mean(values[env_ids]); over all ranks' envs (sum and count all-reduced) with several ranks."""
        if self._dist is None:
            return torch.mean(values[env_ids])
        dev = self.device if self._dist.get_backend() == "nccl" else "cpu"
        t = torch.stack([values[env_ids].double().sum(), torch.tensor(float(len(env_ids)), dtype=torch.float64,
                                                                       device=values.device)]).to(dev)
        self._dist.all_reduce(t)
        return (t[0] / t[1]).float().to(values.device)

    def update_command_curriculum(self, env_ids, cfg, episode_sums=None):
        """_update_command_curriculum_uniform (legged_robot.py:851-880)."""
        c = cfg.commands
        if c.command_curriculum and (self.common_step_counter % cfg.env.max_episode_length == 0):
            if self.reward_scales.get("tracking_lin_vel", 0) > 0:
                m = self._ids_mean(self.episode_sums["tracking_lin_vel"], env_ids) / cfg.env.max_episode_length
                if m > c.forward_curriculum_threshold * self.reward_scales["tracking_lin_vel"]:
                    cfg.command_ranges["lin_vel_x"][0] = np.clip(cfg.command_ranges["lin_vel_x"][0] - 0.2,
                                                                 -c.max_reverse_curriculum, 0.0)
                    cfg.command_ranges["lin_vel_x"][1] = np.clip(cfg.command_ranges["lin_vel_x"][1] + 0.2, 0.0,
                                                                 c.max_forward_curriculum)
        if c.yaw_command_curriculum and (self.common_step_counter % cfg.env.max_episode_length == 0):
            if self.reward_scales.get("tracking_ang_vel", 0) > 0:
                m = self._ids_mean(self.episode_sums["tracking_ang_vel"], env_ids) / cfg.env.max_episode_length
                if m > c.yaw_curriculum_threshold * self.reward_scales["tracking_ang_vel"]:
                    cfg.command_ranges["ang_vel_yaw"][0] = np.clip(cfg.command_ranges["ang_vel_yaw"][0] - 0.2,
                                                                   -c.max_yaw_curriculum, 0.0)
                    cfg.command_ranges["ang_vel_yaw"][1] = np.clip(cfg.command_ranges["ang_vel_yaw"][1] + 0.2, 0.0,
                                                                   c.max_yaw_curriculum)

    def reset_evaluation_envs(self):
        """legged_robot.py:204-225: log the evaluation batch (mean of each eval env's first finished episode,
        or its running sum if none finished), advance the eval command curriculum, reset every eval env."""
        if self.eval_cfg is None:
            return
        ids = torch.arange(self.num_train_envs, self.num_envs, device=self.device)
        ep = self.extras.get("eval/episode")
        if ep is None:
            ep = self.extras["eval/episode"] = {}
        for k in self.episode_sums_eval:
            unset = ids[self.episode_sums_eval[k][ids] == -1]
            self.episode_sums_eval[k][unset] = self.episode_sums[k][unset]
            s = self.episode_sums_eval[k]
            ep["rew_" + k] = torch.mean(s[s != -1])
        self.update_command_curriculum(ids, self.eval_cfg, self.episode_sums_eval)
        self.reset_idx(ids)
        for k in self.episode_sums_eval:
            self.episode_sums_eval[k] = -torch.ones(self.num_envs, device=self.device)

    # ---- gymapi-style setters (data is already in place when written through the views) ----
    def set_actor_root_state_tensor_indexed(self, root_states, env_ids):
        ids = torch.as_tensor(env_ids, device=self.device).to(torch.int32).contiguous()
        src = root_states.contiguous()
        _abi.check(self._L.lrl_sim_set_root_state_indexed(self._sim, C.c_void_p(src.data_ptr()),
                                                          C.c_void_p(ids.data_ptr()), C.c_int32(len(ids)),
                                                          self._stream()))

    def set_dof_state_tensor_indexed(self, dof_pos, dof_vel, env_ids):
        ids = torch.as_tensor(env_ids, device=self.device).to(torch.int32).contiguous()
        p, v = dof_pos.contiguous(), dof_vel.contiguous()
        _abi.check(self._L.lrl_sim_set_dof_state_indexed(self._sim, C.c_void_p(p.data_ptr()), C.c_void_p(v.data_ptr()),
                                                         C.c_void_p(ids.data_ptr()), C.c_int32(len(ids)),
                                                         self._stream()))

    def shift_history(self):
        _abi.check(self._L.lrl_sim_shift_history(self._sim, self._stream()))

    # ---- recording hooks used by Runner.log_video (rendering is out of scope) ----
    def start_recording(self):
        self.record_now = True

    def start_recording_eval(self):
        pass

    def pause_recording(self):
        self.record_now = False

    def pause_recording_eval(self):
        pass

    def get_complete_frames(self):
        return []

    def get_complete_frames_eval(self):
        return []


VelocityTrackingEasyEnv = LeggedRobotEnv
