"""bench.py's secondary line (configs[2]: 4096 Go1 envs on the curriculum trimesh, upstream resets) alone, for a
rocprofv3 kernel trace.  usage: python scripts/sec_trace.py [iters]"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rapid-locomotion-rl_amd"))
spec = importlib.util.spec_from_file_location("bench_sec", os.path.join(ROOT, "bench.py"))
b = importlib.util.module_from_spec(spec)
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
sys.argv = [sys.argv[0]]
spec.loader.exec_module(b)
out = b.bench_go1_rough("cuda:0", iters=iters, warmup=2)
print(json.dumps({k: out[k] for k in ("env_steps_per_s", "ppo_iters_per_s", "env_step_kernel_ms")}), flush=True)
