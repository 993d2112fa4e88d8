"""Run-to-run determinism probe of the configs[3] rollout (tests/test_configs_gpu.py::_iteration, 4096 Mini Cheetah
envs, 24 steps, rollout only): the same rollout repeated in one process, then with every CU's LDS filled with a
pattern before each env step (scripts/liblds_poison.so), each compared with the first run key by key; a mismatch is
located by (step, env).  usage: python scripts/determinism_probe.py [repeats] [patterns...]"""
import ctypes as C
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from lrl import _abi  # noqa: E402
from ranks import init_rank  # noqa: E402
import test_configs_gpu as T  # noqa: E402


def compare(tag, a, b):
    bad = False
    for k in T.STORE_KEYS + ["root", "dof_pos", "dof_vel", "contact", "hist", "origins"]:
        x, y = a[k], b[k]
        ne = x != y
        if k == "advantages" or not ne.any():
            continue
        bad = True
        idx = np.argwhere(ne)
        if k in T.STORE_KEYS:
            steps = np.unique(idx[:, 0])
            envs = np.unique(idx[:, 1])
            print(f"  {tag} {k}: {ne.sum()} differ, steps {steps[:12].tolist()} envs {envs[:24].tolist()}"
                  f" ({len(envs)} envs) max|d| {np.abs(x - y)[ne].max():.3e}", flush=True)
        else:
            envs = np.unique(idx[:, 0])
            print(f"  {tag} {k}: {ne.sum()} differ, envs {envs[:24].tolist()} ({len(envs)} envs)", flush=True)
    print(f"{tag}: {'DIFFERS' if bad else 'identical'}", flush=True)
    return bad


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    pats = [int(p, 0) for p in sys.argv[2:]] if len(sys.argv) > 2 else [0x7FC00000, 0x47000000]
    init_rank(0, 1, 0)
    tmp = tempfile.mkdtemp()
    ref = T._iteration("mc", 0, 1, tmp, T.N_BENCH, True, True)
    print("reference run done", flush=True)
    any_bad = False
    for r in range(reps):
        any_bad |= compare(f"repeat{r}", T._iteration("mc", 0, 1, tmp, T.N_BENCH, True, True), ref)
    P = C.CDLL(os.path.join(ROOT, "scripts", "liblds_poison.so"))
    P.lds_poison.restype = C.c_int
    P.lds_poison.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p]
    sink = torch.zeros(256 * 8, dtype=torch.int32, device="cuda:0")
    L = _abi.lib()
    # every C-ABI entry point include/lrl.h declares: the LDS is poisoned on the current stream before each call
    import re
    names = sorted(set(re.findall(r"\b(lrl_\w+)\s*\(", open(os.path.join(ROOT, "include", "lrl.h")).read())))
    origs = {nm: getattr(L, nm) for nm in names if hasattr(L, nm)}
    for pat in pats:
        def wrap(nm, _p=pat):
            o = origs[nm]

            def call(*a):
                st = torch.cuda.current_stream().cuda_stream
                assert P.lds_poison(_p, sink.data_ptr(), C.c_void_p(st)) == 0
                return o(*a)
            return call
        for nm in origs:
            setattr(L, nm, wrap(nm))
        try:
            any_bad |= compare(f"poison{pat:#x}", T._iteration("mc", 0, 1, tmp, T.N_BENCH, True, True), ref)
        finally:
            for nm, o in origs.items():
                setattr(L, nm, o)
    assert int(sink.sum()) == 0
    # timing perturbation: another process keeps the GPU busy with GEMMs while the rollout runs (as the 2-rank
    # sharding test's ranks share the card)
    import subprocess
    load = subprocess.Popen([sys.executable, "-c",
                             "import torch,time\n"
                             "a=torch.randn(4096,4096,device='cuda:0');t=time.time()\n"
                             "while time.time()-t<90:\n  b=a@a\n  torch.cuda.synchronize()\n"])
    try:
        for r in range(reps):
            any_bad |= compare(f"loaded{r}", T._iteration("mc", 0, 1, tmp, T.N_BENCH, True, True), ref)
    finally:
        load.kill()
        load.wait()
    print("RESULT", "nondeterministic" if any_bad else "deterministic", flush=True)


if __name__ == "__main__":
    main()
