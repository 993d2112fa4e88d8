#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/probe/r6zb.sh && bash scripts/probe/r6za.sh
