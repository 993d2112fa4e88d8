"""Which side of the sharding comparison varies: the 1 x 4096 rollout twice and the 2 x 2048 rollout twice (fresh
processes each), each pair compared key by key (tests/test_configs_gpu.py::_rank_worker, rollout only, fork resets)."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))

if __name__ == "__main__":
    import torch.multiprocessing as mp
    import test_configs_gpu as T
    n = T.N_BENCH
    keys = T.STORE_KEYS + ["root", "dof_pos", "dof_vel", "contact", "hist", "origins"]

    def one():
        mgr = mp.Manager()
        d = mgr.dict()
        with tempfile.TemporaryDirectory() as tmp:
            mp.spawn(T._rank_worker, args=(1, 0, "mc", tmp, d, n, True, True), nprocs=1, join=True)
        return {k: d[0][k] for k in keys}

    def two():
        mgr = mp.Manager()
        d = mgr.dict()
        with tempfile.TemporaryDirectory() as tmp:
            mp.spawn(T._rank_worker, args=(2, T._port(), "mc", tmp, d, n // 2, True, True), nprocs=2, join=True)
        return {k: np.concatenate([d[0][k], d[1][k]], axis=1 if k in T.STORE_KEYS else 0) for k in keys}

    def cmp(tag, a, b):
        bad = [k for k in keys if not np.array_equal(a[k], b[k])]
        envs = set()
        for k in bad:
            ne = a[k] != b[k]
            idx = np.argwhere(ne)
            envs |= set((idx[:, 1] if k in T.STORE_KEYS else idx[:, 0]).tolist())
        print(tag, "identical" if not bad else f"differ in {bad}, envs {sorted(envs)[:20]} ({len(envs)})", flush=True)
    for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
        o1, o2, t1, t2 = one(), one(), two(), two()
        cmp(f"[{r}] one vs one", o1, o2)
        cmp(f"[{r}] two vs two", t1, t2)
        cmp(f"[{r}] one vs two", o1, t1)
