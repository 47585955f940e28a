#!/bin/bash
# both: sharded-vs-unsharded C5 traces (r03ab), then the final-build tile counters (r03aa)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 700 bash scripts/gpu_r03ab.sh || exit 1
timeout -k 10 700 bash scripts/gpu_r03aa.sh || exit 1
