# GPU box: fused stage A at U = 2 (LRS_A_FUSED_U2=1) against U = 1, north-star leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do for v in 1 0; do
  echo "U2=$v"; LRS_A_FUSED_U2=$v timeout -k 10 200 python -u scripts/leg_probe.py g81 10 || exit 1
done; done
