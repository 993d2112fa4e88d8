"""A/B of bench.py's secondary line (BASELINE configs[2]: 4096 Go1 envs on the curriculum trimesh, upstream resets)
for the tree on PYTHONPATH (scripts/ab_tree.sh): one JSON line.  usage: python scripts/ab_secondary.py <tag> [iters]"""
import importlib.util
import json
import os
import sys

tag = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 8
tree = os.path.dirname(os.path.dirname(os.path.abspath(sys.modules["lrl"].__file__))) if "lrl" in sys.modules else None
import lrl  # noqa: E402  (from PYTHONPATH)
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(lrl.__file__))))
spec = importlib.util.spec_from_file_location("bench_ab", os.path.join(root, "bench.py"))
b = importlib.util.module_from_spec(spec)
sys.argv = [sys.argv[0]]
spec.loader.exec_module(b)
out = b.bench_go1_rough("cuda:0", iters=iters, warmup=2)
print(json.dumps({"tag": tag, "lrl": os.path.dirname(lrl.__file__), **{k: out[k] for k in ("env_steps_per_s", "ppo_iters_per_s", "env_step_kernel_ms")}}), flush=True)
