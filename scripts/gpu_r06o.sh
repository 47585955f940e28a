# GPU box: the fused stage A with its own grid sizing -- tests of the bandwidth kernels, probes of
# the north-star and at-scale legs, then the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bw_kernels.py > gpurun_out/r06o_bw.txt 2>&1; echo "bw tests rc $?"; tail -n 2 gpurun_out/r06o_bw.txt
for leg in g81 torus2000; do timeout -k 10 200 python -u scripts/leg_probe.py $leg 10 || exit 1; done
timeout -k 10 900 python -u bench.py > gpurun_out/r06o_bench.json.log 2> gpurun_out/r06o_bench.err; echo "bench rc $?"
