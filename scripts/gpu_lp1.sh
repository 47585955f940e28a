# GPU box: the LP cone, the comm-recording and --oracleRankNaive tests, then shmup4 through the CLI
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_steps.py -k "mc_lp60" > gpurun_out/lp1_steps.txt 2>&1; echo "steps rc $?"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_lp.py tests/test_gpu_shard_comm.py "tests/test_gpu_cli.py::test_oracle_rank_naive_matches_reference" > gpurun_out/lp1_pytest.txt 2>&1; echo "pytest rc $?"
grep -E "passed|failed|PASS|FAIL|Error|shmup4:" gpurun_out/lp1_steps.txt gpurun_out/lp1_pytest.txt | tail -40
