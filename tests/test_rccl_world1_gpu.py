"""The update's collectives through RCCL on the one GPU of a test box ("no nccl collective has ever run").
RCCL refuses two ranks on one GPU, so scripts/rccl_world1.py runs one native update inside a one-rank `nccl` group
with LRL_FORCE_COLLECTIVES=1: every collective a multi-GPU update issues (advantage statistics, the flat policy
gradient + KL slot per optimiser step, the adaptation gradient per substep) goes through RCCL on the update's own
device buffers and streams, each reducing over the one rank.  The same under `gloo` (host-staged) must give the same
bits, and both must match the update without collectives to fp32 rounding (they normalise the advantages from
all-reduced sums instead of in one pass)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_update_collectives_run_through_rccl(tmp_path):
    from lrl.ppo.ppo import PPO_Args
    runs = {}
    for backend in ("none", "nccl", "gloo"):
        out = tmp_path / f"{backend}.npz"
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
                   LOCAL_RANK="0", LRL_FORCE_COLLECTIVES="1")
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_world1.py"), backend, str(out)], env=env,
                       check=True, timeout=240)
        runs[backend] = np.load(out)
    steps = PPO_Args.num_learning_epochs * PPO_Args.num_mini_batches
    want = 1 + steps * (1 + PPO_Args.num_adaptation_module_substeps)  # advantage stats, then per optimiser step
    assert len(runs["none"]["sizes"]) == 0
    for b in ("nccl", "gloo"):
        assert len(runs[b]["sizes"]) == want, (b, runs[b]["sizes"])
        assert runs[b]["sizes"][0] == 3
        # RCCL reduces the device buffers in place; gloo gets the host-staged copies (lrl/ppo/ppo.py _all_reduce_)
        assert runs[b]["on_device"].all() if b == "nccl" else not runs[b]["on_device"].any(), (b, runs[b]["on_device"])
    for k in ("flat", "adv", "losses"):
        np.testing.assert_array_equal(runs["nccl"][k], runs["gloo"][k])
    np.testing.assert_allclose(runs["nccl"]["adv"], runs["none"]["adv"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(runs["nccl"]["flat"], runs["none"]["flat"], rtol=0, atol=1e-5)
