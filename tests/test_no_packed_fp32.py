"""liblrl.so carries no packed-FP32 VALU instructions.

With them, lanes 48-63 of the plane env kernel's wave took results that depended on another process's kernels running
on the same GPU (the 1 x 4096 / 2 x 2048 rollouts of tests/test_configs_gpu.py diverged in envs of that lane group, the
replay check in scripts/sharding_replay.py caught the step itself changing; with the same kernel built without
v_pk_fma / v_pk_mul / v_pk_add_f32 and v_pk_mov_b32, 20 of 20 two-rank rollouts replayed and matched).  The Makefile
builds every kernel with the feature off; this test reads the gfx950 code objects out of the built library and checks
that none of those instructions came back (a build-flag regression would otherwise pass every single-process test)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rapid-locomotion-rl_amd", "csrc", "liblrl.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PACKED = ("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_pk_mov_b32")


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(os.path.join(LLVM, "llvm-objdump"))),
                    reason="liblrl.so or the ROCm LLVM tools are absent")
def test_library_has_no_packed_fp32_instructions(tmp_path):
    fat = tmp_path / "fat.bin"
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", LIB])
    data = fat.read_bytes()
    starts = []
    i = data.find(MAGIC)
    while i >= 0:
        starts.append(i)
        i = data.find(MAGIC, i + 1)
    assert starts, "no offload bundle in .hip_fatbin"
    n_kernels, found = 0, {}
    for k, s in enumerate(starts):  # one bundle per translation unit
        chunk = tmp_path / f"b{k}.bin"
        chunk.write_bytes(data[s:starts[k + 1] if k + 1 < len(starts) else len(data)])
        co = tmp_path / f"co{k}.o"
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--unbundle",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={chunk}", f"--output={co}"])
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", str(co)], capture_output=True, text=True,
                             check=True).stdout
        n_kernels += dis.count(">:\n")
        for op in PACKED:
            c = dis.count(op + " ")
            if c:
                found[op] = found.get(op, 0) + c
    assert n_kernels > 20, n_kernels  # (the env, GEMM, PPO and aux kernels were all looked at)
    assert not found, found
