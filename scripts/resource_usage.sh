#!/bin/bash
# Code-object resource notes of every kernel (VGPR / AGPR / SGPR spills / scratch / occupancy / LDS), from the
# compiler's kernel-resource-usage remarks on the same flags as the Makefile.  Runs on the CPU (cross-compile).
# usage: bash scripts/resource_usage.sh > profiles/<tag>_resources.txt
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT/rapid-locomotion-rl_amd/csrc"
for f in lrl_env.hip lrl_env_flat.hip lrl_aux.hip lrl_gae.hip lrl_gemm.hip lrl_ppo.hip lrl_curriculum_dev.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast-honor-pragmas --cuda-device-only \
    -Rpass-analysis=kernel-resource-usage -c "$f" -o /tmp/lrl_res_$$.o 2>&1 |
    sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
    awk -v F="$f" '/^Function Name:/ {printf "\n%s %s", F, $3; next}
                   /^(VGPRs|AGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill|LDS Size)/ {printf " | %s", $0}'
done
echo
rm -f /tmp/lrl_res_$$.o
