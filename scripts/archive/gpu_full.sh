#!/bin/bash
# the whole GPU suite (as the driver runs it at round end), log under gpurun_out/<tag>/
tag=${1:-full}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/$tag
timeout -k 10 1150 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread \
  > gpurun_out/$tag/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/$tag/pytest.log
exit $rc
