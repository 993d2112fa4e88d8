"""CPU-side checks of the C-ABI boundary: liblrl.so loads and exports every function that
include/lrl.h declares; the ctypes struct mirror has the C layout.  No compute calls."""
import ctypes as C
import os
import re
import subprocess

import pytest

from lrl import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "lrl.h")


def _declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lrl_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_abi.LIB_PATH):
        pytest.skip("liblrl.so not built")
    lib = C.CDLL(_abi.LIB_PATH)
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.lrl_abi_version() == 6


def test_library_matches_the_sources_beside_it():
    """Stale-binary guard: the hash baked into liblrl.so (csrc/Makefile SRC_HASH) equals the hash of the tree's
    sources, and the loader refuses a library whose hash differs."""
    if not os.path.exists(_abi.LIB_PATH):
        pytest.skip("liblrl.so not built")
    lib = C.CDLL(_abi.LIB_PATH)
    lib.lrl_build_hash.restype = C.c_char_p
    assert lib.lrl_build_hash().decode() == _abi.source_hash()
    assert _abi.lib() is not None
    saved, _abi._lib = _abi._lib, None
    real = _abi.source_hash
    try:
        _abi.source_hash = lambda: "0" * 16
        with pytest.raises(RuntimeError, match="other sources"):
            _abi.lib()
    finally:
        _abi.source_hash, _abi._lib = real, saved


def test_struct_layout_matches_header():
    code = r"""
#include <stdio.h>
#include <stddef.h>
#include "lrl.h"
int main(){printf("%zu %zu %zu %zu %zu %zu\n", sizeof(lrl_model), sizeof(lrl_env_params), sizeof(lrl_tensor),
 offsetof(lrl_env_params, noise_vec), offsetof(lrl_env_params, max_episode_length), sizeof(lrl_rollout_store));
printf("%zu %zu %zu %zu %zu %zu\n", sizeof(lrl_ppo_net), offsetof(lrl_ppo_net, total), sizeof(lrl_ppo_batch),
 offsetof(lrl_ppo_batch, batch), sizeof(lrl_ppo_hparams), sizeof(lrl_ppo_ctrl));
printf("%zu %zu\n", offsetof(lrl_ppo_batch, hist_ld), offsetof(lrl_rollout_store, hist_ld));
printf("%zu %zu %zu\n", sizeof(lrl_dev_curriculum), offsetof(lrl_dev_curriculum, nz), offsetof(lrl_dev_curriculum, draws));
return 0;}
"""
    exe = "/tmp/lrl_layout_check"
    src = exe + ".c"
    open(src, "w").write(code)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, src])
    out = [int(x) for x in subprocess.check_output([exe]).split()]
    assert out == [C.sizeof(_abi.LrlModel), C.sizeof(_abi.LrlEnvParams), C.sizeof(_abi.LrlTensor),
                   _abi.LrlEnvParams.noise_vec.offset, _abi.LrlEnvParams.max_episode_length.offset,
                   C.sizeof(_abi.LrlRolloutStore), C.sizeof(_abi.LrlPpoNet), _abi.LrlPpoNet.total.offset,
                   C.sizeof(_abi.LrlPpoBatch), _abi.LrlPpoBatch.batch.offset, C.sizeof(_abi.LrlPpoHparams),
                   _abi.PPO_CTRL_BYTES, _abi.LrlPpoBatch.hist_ld.offset, _abi.LrlRolloutStore.hist_ld.offset,
                   C.sizeof(_abi.LrlDevCurriculum), _abi.LrlDevCurriculum.nz.offset, _abi.LrlDevCurriculum.draws.offset]


def test_product_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from lrl.env import LeggedRobotEnv
    with pytest.raises(RuntimeError):
        LeggedRobotEnv("cuda:0")
