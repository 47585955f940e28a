# GPU box: bitwise test of the restructured bandwidth-regime kernels, A/B on the legs, GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bw_kernels.py > gpurun_out/r06i_bw.txt 2>&1; rc=$?; echo "bw rc $rc"
grep -E "PASS|FAIL|Error|assert" gpurun_out/r06i_bw.txt | head -30
[ $rc -eq 0 ] || exit 1
O=gpurun_out/r06i_ab.txt; : > $O
for v in 1 0 1 0; do
  for leg in g81 torus2000; do
    echo "LRS_BW=$v $leg" >> $O
    LRS_BW_A=$v LRS_BW_B=$v timeout -k 10 200 python -u scripts/leg_probe.py $leg 10 >> $O 2>&1 || { echo "probe rc $?"; exit 1; }
  done
done
grep -E "LRS_BW|it_s" $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r06i_pytest_gpu.txt 2>&1; echo "pytest rc $?"
tail -n 5 gpurun_out/r06i_pytest_gpu.txt
