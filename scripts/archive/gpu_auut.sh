#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for bs in 256 512 1024; do for u in 1 2 4; do
  echo "BS=$bs U=$u"; LRS_DIAG_BS=$bs LRS_DIAG_U=$u timeout -k 10 120 python -u scripts/auut_probe.py || exit $?
done; done
