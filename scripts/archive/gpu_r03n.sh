#!/bin/bash
# sharded 2-D tiles: new tests + the tile / shard suites, then the headline / SQ probe (r03m)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03n; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -rfE --timeout 600 --timeout-method thread tests/test_gpu_shard_tiles.py \
  tests/test_gpu_shard.py tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py "tests/test_gpu_steps.py" > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r03m.sh
