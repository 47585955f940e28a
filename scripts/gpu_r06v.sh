# GPU box: k_tile_a with its next step's tiles fetched under the sums (main) against the fetch
# right before its barrier (old: -DLRS_TILE_A_PIPE=0), C5 leg; then the C5 step tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do for v in main old; do
  if [ $v = main ]; then L=""; else L=$GRAFT_REPO_ROOT/ltr-lowrank-sdp_amd/_build/liblrsdp_old.so; fi
  echo "lib $v"; LRS_LIB=$L timeout -k 10 300 python -u scripts/leg_probe.py c5 10 || exit 1
done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c5_steps.py > gpurun_out/r06v_c5_steps.txt 2>&1; echo "c5 steps rc $?"; tail -n 2 gpurun_out/r06v_c5_steps.txt
