# GPU box: stage A fused in the bandwidth regime (LRS_A_FUSED=1: k_it_a MODE 0 at U = 1) against
# the split form, north-star and at-scale legs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06m_ab.txt; : > $O
for r in 1 2; do
  for v in 1 0; do
    for leg in g81 torus2000; do
      echo "LRS_A_FUSED=$v $leg" >> $O
      LRS_A_FUSED=$v timeout -k 10 200 python -u scripts/leg_probe.py $leg 10 >> $O 2>&1 || { echo "probe rc $?"; exit 1; }
    done
  done
done
python3 - <<'PY'
import json
cur=None
for l in open("gpurun_out/r06m_ab.txt"):
    if l.startswith("LRS_"): cur=l.strip()
    elif l.startswith("{"):
        d=json.loads(l); print(cur, "stages", [round(x,1) for x in d["stage_us"]], "it/s", round(d["it_s"]))
PY
