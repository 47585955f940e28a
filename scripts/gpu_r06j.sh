# GPU box: bitwise test of the restructured kernels (opaque diagonal), then A/B of stage A's
# options (k_bw_a2, MODE 1 first-row prefetch) with k_bw_b on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bw_kernels.py > gpurun_out/r06j_bw.txt 2>&1; rc=$?; echo "bw rc $rc"
grep -E "PASS|FAIL|Error|assert" gpurun_out/r06j_bw.txt | head -30
# (bitwise gate reported above)
O=gpurun_out/r06j_ab.txt; : > $O
for r in 1 2; do
  for cfg in "0 1" "0 0" "1 1"; do
    set -- $cfg
    for leg in g81 torus2000; do
      echo "LRS_BW_A=$1 LRS_A1_PRE=$2 $leg" >> $O
      LRS_BW_A=$1 LRS_A1_PRE=$2 timeout -k 10 200 python -u scripts/leg_probe.py $leg 10 >> $O 2>&1 || { echo "probe rc $?"; exit 1; }
    done
  done
done
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06j_ab.txt"):
    if l.startswith("LRS_"): cur=l.strip()
    elif l.startswith("{"):
        d=json.loads(l); print(cur, "stages", [round(x,1) for x in d["stage_us"]], "it/s", round(d["it_s"]))
PY
