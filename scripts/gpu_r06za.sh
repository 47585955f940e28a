# GPU box: Cardano's cube roots as cbrt -- GPU suite, G67 A/B against the pow build, theta A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r06za_pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc $rc"; tail -n 6 gpurun_out/r06za_pytest_gpu.txt
timeout -k 10 400 python -u scripts/lat_ab.py pow main > gpurun_out/r06za_lat_ab.txt 2>&1; echo "lat rc $?"; cat gpurun_out/r06za_lat_ab.txt
timeout -k 10 400 python -u scripts/small_lib_ab.py theta3 > gpurun_out/r06za_theta_ab.txt 2>&1; echo "theta rc $?"; cat gpurun_out/r06za_theta_ab.txt
