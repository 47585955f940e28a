# GPU box: k_bw_a2 (bandwidth-regime SDDMM half, four memory trips a row) against k_it_a MODE 2
# (LRS_BW_A=0), k_bw_b on, north-star and at-scale legs; then the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06h_ab.txt; : > $O
for v in 1 0 1 0; do
  for leg in g81 torus2000; do
    echo "LRS_BW_A=$v $leg" >> $O
    LRS_BW_A=$v timeout -k 10 200 python -u scripts/leg_probe.py $leg 10 >> $O 2>&1 || { echo "probe rc $?"; exit 1; }
  done
done
grep -E "LRS_BW_A|it_s" $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r06h_pytest_gpu.txt 2>&1; echo "pytest rc $?"
tail -n 5 gpurun_out/r06h_pytest_gpu.txt
