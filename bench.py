"""Benchmark: env-steps/s for 4096 Mini Cheetah envs per GPU (weak scaling) + PPO iters/s.

One timed "step" = one PPO iteration of mini_gym_learn's Runner.learn (mini_gym_learn/ppo/
__init__.py:123-242): 24 rollout steps (fused policy kernel + fused env-step kernel per step),
GAE, then 5 epochs x 4 minibatches of the PPO + adaptation update.  value = all ranks' env-steps
(N_gpu x 4096 x 24 x K) / max-over-ranks wall time of the K timed iterations.

  python bench.py [--gpus N --steps K --warmup W]           (N > 1: under torch.distributed.run)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ENVS_PER_GPU = 4096
B_ENV = 1325            # algorithmic HBM bytes per env-step; history shift adds 4872
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TF = 157.3  # dense fp32 MFMA peak (v_mfma_f32_32x32x2_f32, MI355X_MICROARCH.md)
# The update's fp32 products run on the bf16 MFMA with an exact 3-way operand split and six products per k-step
# (csrc/lrl_gemm.hip gemm_x6_kernel, fp32-class error): their bound is the dense bf16 peak / 6 per fp32 FLOP
MFMA_BF16_PEAK_TF = 2500.0
X6_PEAK_TF = MFMA_BF16_PEAK_TF / 6


def pmc_traffic(*kernels):
    """HBM bytes per launch of the first of ``kernels`` (symbol, or symbol@grid) found in the committed PMC summary
    profiles/PMC_CURRENT names (else the newest by name: profiles/r*_pmc.json, written by scripts/gpu_profile.sh +
    scripts/pmc_summary.py from separate rocprofv3 --pmc passes)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    cur = os.path.join(ROOT, "profiles", "PMC_CURRENT")  # the summary of the tree's own kernels, when named
    if os.path.exists(cur):
        with open(cur) as f:
            named = os.path.join(ROOT, "profiles", f.read().strip())
        if os.path.exists(named):
            files = [p for p in files if p != named] + [named]
    for path in reversed(files):
        with open(path) as f:
            table = json.load(f)["kernels"]
        for kernel in kernels:
            k = table.get(kernel)
            if k:
                return k["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def env_kernel_timing(env, start):
    """HIP events around each env-kernel launch of lrl_sim_step, on its launch stream (LeggedRobotEnv.kernel_timing;
    the history shift launched before it is outside): start=True begins recording, start=False returns the mean ms."""
    r = env.kernel_timing(start)
    return None if start else r[0]


def _cpu_info():
    """(threads this process may use, CPU model) — the GPU box's CPU share is its OMP_NUM_THREADS (16), nproc shows
    the whole machine."""
    avail = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return (min(avail, omp) if omp > 0 else avail), avail, model


def cpu_baseline(env_seconds=4.0):
    """CPU baseline on this box's host cores, on bounded samples of the same workload:
    * a whole PPO iteration of configs[1] (4096 Mini Cheetah envs x 24 steps + GAE + the 5 x 4 minibatch update):
      the env is the oracle's float + OpenMP build over all usable cores (oracle/cpu_env.py), the policy and update
      the reference's torch PPO math on the CPU (lrl.ppo with fused=False, torch threads = the same cores) —
      ``value`` is its env-steps/s, the unit of the headline;
    * env-only stepping rates of the same CPU env with all usable cores and with one core (random actions).
    The reference's own Isaac Gym CPU pipeline (PhysX CPU, num_threads=10) is proprietary and absent."""
    from oracle.cpu_env import CpuVecEnv, cpu_compute_returns
    from lrl.ppo import runner as R
    threads, avail, model = _cpu_info()
    prev_threads = torch.get_num_threads()

    def env_rate(n, th):
        env = CpuVecEnv(n, threads=th)
        rng = np.random.default_rng(1)
        a = torch.from_numpy((rng.normal(size=(n, 12)) * 0.3).astype(np.float32))
        env.step(a)
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < env_seconds:
            env.step(a)
            steps += 1
        return n * steps / (time.perf_counter() - t0), steps
    env_all, n_all = env_rate(ENVS_PER_GPU, threads)
    env_one, n_one = env_rate(256, 1)
    torch.set_num_threads(threads)
    env = CpuVecEnv(ENVS_PER_GPU, threads=threads)
    runner = R.Runner(env, device="cpu", seed=1234)
    runner.alg.storage.compute_returns = cpu_compute_returns(runner.alg.storage)
    t0 = time.perf_counter()
    runner.learn(1)
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev_threads)
    steps_iter = ENVS_PER_GPU * R.RunnerArgs.num_steps_per_env
    return dict(value=round(steps_iter / dt, 1), unit="env-steps/s", cores=threads, kind="port",
                ppo_iter_s=round(dt, 3),
                env_only_all_cores_env_steps_per_s=round(env_all, 1),
                env_only_1_core_env_steps_per_s=round(env_one, 1),
                cpu_model=model, threads_used=threads, cpus_visible_machine=os.cpu_count(), cpus_in_affinity_mask=avail,
                cores_note=(f"cores = the {threads} threads every leg ran on (this box's CPU share, OMP_NUM_THREADS); "
                            "the affinity mask shows the whole machine's CPUs, which this job may not use"),
                sample=(f"one PPO iteration of {ENVS_PER_GPU} Mini Cheetah envs x {R.RunnerArgs.num_steps_per_env} steps "
                        f"+ update ({dt:.1f} s; env: oracle/lrl_oracle.c float + OpenMP, {threads} threads; policy / "
                        f"update: torch CPU, {threads} threads); env-only: {ENVS_PER_GPU} envs x {n_all} steps on "
                        f"{threads} threads, 256 envs x {n_one} steps on 1 thread ({env_seconds:.0f} s each). The "
                        "reference's Isaac Gym CPU pipeline is proprietary and absent (BASELINE.md §3)"))


def bench_go1_rough(dev, iters=6, warmup=2):
    """Secondary line, BASELINE configs[2]: 4096 Go1 envs on the curriculum trimesh (stairs, slopes, obstacles,
    stepping stones; terrain curriculum) with the upstream reset path (legacy_fork=False: time-outs, reset_idx
    inside step, grid-adaptive command curriculum) — full PPO iterations, same timing rules as the headline."""
    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    from lrl.history import HistoryWrapper
    from lrl.ppo import runner as R
    cfg = lcfg.make_cfg()
    lcfg.config_go1(cfg)
    cfg.env.num_envs = ENVS_PER_GPU
    cfg.terrain.mesh_type = "trimesh"
    cfg.terrain.terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]  # legged_robot_config.py:57
    cfg.terrain.curriculum = True
    env = HistoryWrapper(LeggedRobotEnv(dev, cfg=cfg, seed=4321, legacy_fork=False))
    runner = R.Runner(env, device=dev, seed=4321)
    runner.learn(warmup, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    env_kernel_timing(env.env, True)
    t0 = time.perf_counter()
    runner.learn(iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    k_ms = env_kernel_timing(env.env, False)
    out = {"workload": "4096 Go1 envs, trimesh rough terrain (curriculum tiles) + terrain curriculum + upstream resets "
                       "with the grid-adaptive command curriculum (BASELINE configs[2])",
           "env_steps_per_s": round(ENVS_PER_GPU * R.RunnerArgs.num_steps_per_env * iters / dt, 1),
           "ppo_iters_per_s": round(iters / dt, 3), "env_step_kernel_ms": round(k_ms, 4), "steps": iters}
    env.env.close()
    return out


WORKLOADS = {
    "mc": lambda w: (f"{w * ENVS_PER_GPU} Mini Cheetah envs flat terrain ({ENVS_PER_GPU} per GPU), PPO teacher policy "
                     f"(BASELINE configs[{1 if w == 1 else 3}])"),
    "go1": lambda w: (f"{w * ENVS_PER_GPU} Go1 envs on the plane ({ENVS_PER_GPU} per GPU), teacher PPO + student "
                      "(adaptation-module) distillation update (BASELINE configs[4] at 2 GPUs)"),
}


# BASELINE.json's metric (the headline, Mini Cheetah); the Go1 workload names its own robot
METRICS = {"mc": "env-steps/sec, 4096 Mini Cheetah envs, 1/2/4/8 MI355X; PPO iters/sec",
           "go1": "env-steps/sec, 4096 Go1 envs per GPU (teacher-student update), 1/2 MI355X; PPO iters/sec"}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """``--gpus N`` without a launcher: start N child processes of this script, one per GPU, with the
    torch.distributed.run environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), relay their output and
    exit with the worst return code.  The parent never touches the GPU (torch.cuda.device_count() does not
    initialise it on this image), so no process that holds a GPU context is replaced or forked."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def init_world(args):
    """Join (or skip) the process group; returns (world, rank, local_rank, backend).  Every rank asserts that the
    world it joined has exactly ``--gpus`` ranks."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # one rank per GPU over RCCL ("nccl"); LRL_DIST_BACKEND=gloo rehearses the multi-rank path on CPU or with
    # several ranks sharing one GPU (ranks then use devices round-robin)
    backend = os.environ.get("LRL_DIST_BACKEND", "nccl")
    # LRL_FORCE_COLLECTIVES=1 at one GPU: a one-rank RCCL group, and the update issues its collectives anyway (each
    # reducing over the one rank) — the N = 1 line with the collectives' call cost in it
    force1 = world == 1 and os.environ.get("LRL_FORCE_COLLECTIVES") == "1" and not args.world_check
    if force1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend, rank=0, world_size=1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
        got = dist.get_world_size()
        assert got == args.gpus, f"rank {rank}: process group has {got} ranks, --gpus {args.gpus}"
    return world, rank, local, backend


def device_identity(local_dev):
    """(host, PCI bus / device id, UUID) of a visible device: what tells two ranks' GPUs apart."""
    import socket
    p = torch.cuda.get_device_properties(local_dev)
    uuid = str(getattr(p, "uuid", ""))
    pci = f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:{getattr(p, 'pci_device_id', 0):02x}"
    return socket.gethostname(), pci, uuid


def check_rank_devices(world, rank, local_dev, backend):
    """Every rank names its device (stderr) and, with RCCL, the ranks gather them: two ranks on one physical GPU is an
    error (RCCL's ring over xGMI needs one rank per GPU; a duplicate would also double-count a GPU in the scaling line).
    Returns the per-rank device list for the JSON line."""
    ident = device_identity(local_dev)
    print(f"[bench rank {rank}/{world}] pid {os.getpid()} cuda:{local_dev} host {ident[0]} pci {ident[1]} "
          f"uuid {ident[2]} backend {backend if world > 1 else None}", file=sys.stderr, flush=True)
    if world == 1:
        return [{"rank": 0, "device": local_dev, "pci": ident[1]}]
    got = [None] * world
    dist.all_gather_object(got, (rank, local_dev, ident))
    devices = [{"rank": r, "device": d, "host": h, "pci": pci, "uuid": u} for r, d, (h, pci, u) in sorted(got)]
    if backend == "nccl":
        seen = {}
        for e in devices:
            key = (e["host"], e["pci"], e["uuid"])
            if key in seen:
                raise SystemExit(f"bench.py: ranks {seen[key]} and {e['rank']} share GPU {key} — one rank per GPU")
            seen[key] = e["rank"]
        if rank == 0:
            print(f"[bench] RCCL world {dist.get_world_size()}: " + ", ".join(f"r{e['rank']}=cuda:{e['device']}"
                                                                              f"@{e['pci']}" for e in devices),
                  file=sys.stderr, flush=True)
    return devices


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the Go1 rough-terrain line (configs[2])")
    ap.add_argument("--workload", choices=["mc", "go1"], default="mc",
                    help="mc: 4096 Mini Cheetah envs per GPU, flat (configs[1] / [3]); go1: 4096 Go1 envs per GPU, "
                         "plane, teacher + student update (configs[4] at --gpus 2)")
    ap.add_argument("--world-check", action="store_true",
                    help="join a gloo process group, print the world every rank sees and exit (no GPU work)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    backend = os.environ.get("LRL_DIST_BACKEND", "nccl")
    if backend == "nccl":
        # the GPU count is checked for the real launch and for --world-check alike (device_count() opens no context)
        ndev = torch.cuda.device_count()
        if args.gpus > ndev:
            print(f"bench.py: --gpus {args.gpus} requested but {ndev} GPU(s) visible", file=sys.stderr)
            raise SystemExit(2)
    if args.world_check:
        os.environ["LRL_DIST_BACKEND"] = "gloo"  # CPU tensors, no device context
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    # RCCL prints a version banner on stdout when its communicator comes up (and libraries may print too): the bench's
    # stdout carries its one JSON line only — fd 1 goes to stderr for the rest of the run, the JSON line to the saved
    # stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world, rank, local, backend = init_world(args)
    if args.world_check:
        seen = torch.tensor([rank], dtype=torch.int64)
        if world > 1:
            ranks = [torch.zeros_like(seen) for _ in range(world)]
            dist.all_gather(ranks, seen)
            seen_ranks = sorted(int(t.item()) for t in ranks)
        else:
            seen_ranks = [0]
        if rank == 0:
            print(json.dumps({"world_size": world, "ranks": seen_ranks, "backend": backend if world > 1 else None,
                              "parallelism": f"dp{world}"}), file=json_out, flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    ndev = max(1, torch.cuda.device_count())
    local_dev = local % ndev
    torch.cuda.set_device(local_dev)
    dev = f"cuda:{local_dev}"
    devices = check_rank_devices(world, rank, local_dev, backend)

    from lrl import config as lcfg
    from lrl.env import LeggedRobotEnv
    from lrl.history import HistoryWrapper
    from lrl.ppo import runner as R

    cfg = lcfg.make_cfg()
    (lcfg.config_go1 if args.workload == "go1" else lcfg.config_mini_cheetah)(cfg)
    cfg.env.num_envs = ENVS_PER_GPU
    R.RunnerArgs.save_interval = 0
    R.RunnerArgs.log_freq = 10 ** 9
    env = HistoryWrapper(LeggedRobotEnv(dev, cfg=cfg, seed=1234, env_offset=rank * ENVS_PER_GPU))
    g = torch.Generator(device=dev).manual_seed(1 + rank)
    cmd = torch.rand(ENVS_PER_GPU, 3, device=dev, generator=g)
    env.env.commands[:, 0] = cmd[:, 0] * 1.2 - 0.6
    env.env.commands[:, 1] = cmd[:, 1] * 1.2 - 0.6
    env.env.commands[:, 2] = cmd[:, 2] * 2.0 - 1.0
    runner = R.Runner(env, device=dev, seed=1234)
    runner.learn(args.warmup, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    env_kernel_timing(env.env, True)
    import ctypes as C
    from lrl import _abi
    _abi.check(_abi.lib().lrl_ppo_timing(1, None, None))  # events around the update's largest GEMM
    t0 = time.perf_counter()
    runner.learn(args.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    g_ms, g_n = C.c_double(0.0), C.c_int64(0)
    _abi.check(_abi.lib().lrl_ppo_timing(0, C.byref(g_ms), C.byref(g_n)))
    if world > 1:
        dist.barrier()
    k_ms = env_kernel_timing(env.env, False)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    # self-contact slot statistics under the bench's own workload (one more, untimed, iteration with the counters on)
    env.env.self_contact_stats(True)
    runner.learn(1)
    torch.cuda.synchronize()
    sc = env.env.self_contact_stats(False)
    sc["env_substeps"] = ENVS_PER_GPU * R.RunnerArgs.num_steps_per_env * 4
    sc["dropped_fraction_of_pairs"] = sc["self_pairs_dropped"] / max(1, sc["self_pairs_in_contact"])
    # env-only rate: the fused step kernel alone, random actions, same env
    a = torch.randn(ENVS_PER_GPU, 12, device=dev) * 0.3
    for _ in range(10):
        env.step(a)
    torch.cuda.synchronize()
    te = time.perf_counter()
    ne = 100
    for _ in range(ne):
        env.step(a)
    torch.cuda.synchronize()
    env_only = ENVS_PER_GPU * ne / (time.perf_counter() - te)

    steps_total = world * ENVS_PER_GPU * R.RunnerArgs.num_steps_per_env * args.steps
    value = steps_total / elapsed
    if rank == 0:
        achieved = B_ENV * ENVS_PER_GPU / (k_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic("lrl::flat::env_step_kernel<false>", "lrl::env_step_kernel<false>")
        # update's largest product: actor/critic layer-2 weight gradient, 2 x (256 x 512) over the minibatch rows
        mb_rows = ENVS_PER_GPU * R.RunnerArgs.num_steps_per_env // 4
        gemm_flop = 2.0 * 2 * 256 * 512 * mb_rows
        gemm_ms = g_ms.value / max(1, g_n.value)
        gemm_tf = gemm_flop / (gemm_ms * 1e-3) / 1e12 if g_n.value else None
        # dW2 has its own symbol (trace tag 1, csrc/lrl_gemm.hip tn_shape_tag: the LDS-DMA x6t kernel since round 4, the
        # x6 kernel in round 3): its PMC row is this launch's traffic
        gemm_kernel = "lrl::gemm_x6t_kernel<128, 1, false>"
        gemm_traffic, gemm_traffic_src = pmc_traffic(gemm_kernel, "lrl::gemm_x6t_kernel<1, false>",
                                                     "lrl::gemm_x6_kernel<128, 128, 3, 4, true, false, 1>")
        # whole iteration against the fp32 MFMA peak: SURVEY.md §8(d)'s 3.92 MFLOP per minibatch row and epoch of
        # the update (5 epochs over the 98,304 rollout rows) + 0.94 MFLOP per rollout row of the act
        rows_iter = ENVS_PER_GPU * R.RunnerArgs.num_steps_per_env
        iter_flop = rows_iter * (5 * 3.92e6 + 0.94e6)
        iter_tf = iter_flop / (elapsed / args.steps) / 1e12
        # distinct physical devices the ranks ran on (a gloo rehearsal puts several ranks on one GPU)
        n_dev = world if backend == "nccl" else min(world, ndev)
        out = {
            "metric": METRICS[args.workload],
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": n_dev, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "dtype_note": ("f32 throughout (the reference's precision); the update's / act's products are fp32 products "
                           "computed on the bf16 MFMA from an exact 3-way split of each fp32 operand (6 products, fp32 "
                           "accumulation; error at the fp32 MFMA's level, DESIGN.md §3)"),
            "config": {"workload": WORKLOADS[args.workload](world),
                       "envs_per_gpu": ENVS_PER_GPU, "global_envs": world * ENVS_PER_GPU,
                       "global_batch_env_steps_per_iter": world * ENVS_PER_GPU * 24,
                       "parallelism": f"dp{world}", "world_size": world,
                       "backend": (backend if dist.is_initialized() else None), "devices": devices,
                       "policy": "ActorCritic 42/18/630->12, random init; teacher PPO + student adaptation update"},
            "ppo_iters_per_s": round(args.steps / elapsed, 3),
            "env_only_env_steps_per_s_per_gpu": round(env_only, 1),
            "env_step_kernel_ms": round(k_ms, 4),
            "self_contact": dict(sc, note="one untimed PPO iteration after the timed ones; a pair without a slot is "
                                          "one PhysX would solve and this solver skips in that sub-step (DESIGN.md §4)"),
            "roofline": {"bound": "hbm", "kernel": "lrl::flat::env_step_kernel<false> (plane ground)", "achieved": round(achieved, 3),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": round(traffic) if traffic else None, "traffic_source": traffic_src,
                         "note": f"algorithmic {B_ENV} B/env-step x {ENVS_PER_GPU} envs per launch (+ the newest history "
                                 f"slot, 168 B/env-step; the older slots move in the separate shift_history_kernel launch "
                                 "before it); the kernel is latency-bound (16 lanes per env = 4 mirrored quads, one single-wave "
                                 "workgroup per 4 envs, 1,024 waves; the slowest wave sets the launch), see DESIGN.md"},
            "roofline_update_gemm": {
                "bound": "mfma", "kernel": f"{gemm_kernel} (dW2: 2 x 256x512, {mb_rows} rows)",
                "achieved": round(gemm_tf, 2) if gemm_tf else None, "peak": round(X6_PEAK_TF, 1),
                "unit": "TFLOP/s", "frac": round(gemm_tf / X6_PEAK_TF, 4) if gemm_tf else None,
                "arithmetic": "fp32 operands split exactly into 3 bf16 parts, 6 bf16 MFMA products per k-step, fp32 "
                              "accumulation (error at the fp32 level, tests/test_gemm_gpu.py); peak = dense bf16 MFMA "
                              f"{MFMA_BF16_PEAK_TF:.0f} TF / 6 (the fp32 MFMA peak is {MFMA_F32_PEAK_TF} TF)",
                "traffic": round(gemm_traffic) if gemm_traffic else None, "traffic_source": gemm_traffic_src,
                "algorithmic_bytes": 4 * (2 * mb_rows * (256 + 512)),
                "launch_ms": round(gemm_ms, 4), "launches": g_n.value,
                "note": "the GEMM family is ~70% of the iteration's GPU time; this is its largest launch "
                        "(split-k partials written to the workspace count in traffic)"},
            "roofline_iteration": {
                "bound": "mfma", "achieved": round(iter_tf, 2), "peak": round(X6_PEAK_TF, 1), "unit": "TFLOP/s",
                "frac": round(iter_tf / X6_PEAK_TF, 4), "flop_per_iteration": iter_flop,
                "note": "SURVEY.md §8(d): 3.92 MFLOP per row and epoch (update) + 0.94 MFLOP per rollout row; "
                        "the env step's work is not counted"},
            "reference_context": {"upstream_example_run_env_steps_per_s": 41176, "upstream_ppo_iters_per_s": 0.429,
                                  "hardware": "unspecified NVIDIA GPU, 4000 envs (BASELINE.md §1)"},
        }
        if world == 1 and not args.no_secondary:
            env.env.close()
            out["secondary"] = bench_go1_rough(dev)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), file=json_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
