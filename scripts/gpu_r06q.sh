# GPU box: k_bw_a (fused stage A, four trips a row) A/B against k_it_a MODE 0 at the default
# 32x2 row layout and at 64x1 (one wave a row: k_bw_a without spills), north-star leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06q_ab.txt; : > $O
for r in 1 2; do
  for cfg in "32x2 0" "32x2 1" "64x1 0" "64x1 1"; do
    set -- $cfg
    echo "LRS_LAYOUT=$1 LRS_BW_A=$2" >> $O
    LRS_LAYOUT=$1 LRS_BW_A=$2 timeout -k 10 200 python -u scripts/leg_probe.py g81 10 >> $O 2>&1 || { echo "probe rc $?"; exit 1; }
  done
done
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06q_ab.txt"):
    if l.startswith("LRS_"): cur=l.strip()
    elif l.startswith("{"):
        d=json.loads(l); print(cur, "stages", [round(x,1) for x in d["stage_us"]], "it/s", round(d["it_s"]))
PY
