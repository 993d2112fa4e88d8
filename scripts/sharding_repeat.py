"""Repeats tests/test_configs_gpu.py::test_rollout_does_not_depend_on_the_gpu_count in one process (an intermittent
mismatch hunt): usage python scripts/sharding_repeat.py <times> <legacy_fork 0|1> <n>"""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))

if __name__ == "__main__":
    import test_configs_gpu as T
    times, lf, n = int(sys.argv[1]), bool(int(sys.argv[2])), int(sys.argv[3])
    fails = 0
    for i in range(times):
        try:
            T.test_rollout_does_not_depend_on_the_gpu_count(lf, n)
            print(f"run {i}: ok", flush=True)
        except AssertionError as e:
            fails += 1
            print(f"run {i}: MISMATCH\n{e}", flush=True)
    print(f"RESULT {fails} of {times} mismatched", flush=True)
