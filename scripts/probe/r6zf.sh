#!/bin/bash
# bench stdout = its one JSON line: plain, with the one-rank RCCL group, and under torch.distributed.run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/r6zf_plain.out 2> gpurun_out/r6zf_plain.err || exit 1
LRL_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/r6zf_rccl1.out 2> gpurun_out/r6zf_rccl1.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/r6zf_run.out 2> gpurun_out/r6zf_run.err || exit 1
wc -l gpurun_out/r6zf_*.out
echo done
