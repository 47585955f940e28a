#!/bin/bash
# Round 4: MFMA-busy counters of the FP64 matrix-core kernels (k_cgemm2: the C5b dense C R
# product; k_gram: the r x r Gram at n = 1e4, r = 128) -- one SQ pass per program, the counter
# list filtered against what rocprofv3 lists on this gfx950 box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04c; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/list.txt 2>&1 || true
grep -o -E "\b(SQ|GRBM)_[A-Z0-9_]*(MFMA|BUSY|GUI_ACTIVE|WAVE_CYCLES)[A-Z0-9_]*\b" $O/list.txt | sort -u > $O/mfma_counters.txt
cat $O/mfma_counters.txt
want="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
pmc=""
for c in $want; do grep -qx "$c" $O/mfma_counters.txt && pmc="$pmc $c"; done
echo "pmc:$pmc"
[ -n "$pmc" ] || { echo "no MFMA counters listed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $pmc --output-format csv -d $O/cg -o run -- python3 -u $R/scripts/c5b_cgemm_probe.py > $O/cg.log 2>&1 || { tail -5 $O/cg.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $pmc --output-format csv -d $O/gr -o run -- python3 -u $R/scripts/gram_probe.py 100 128 > $O/gr.log 2>&1 || { tail -5 $O/gr.log; exit 1; }
cat $O/cg.log $O/gr.log | grep -v "^E20\|^W20"
for p in cg gr; do
  f=$(ls $O/$p/*counter_collection.csv | head -1)
  for c in $pmc; do
    for k in k_cgemm2 k_gram; do python3 $R/scripts/pmc_sum.py $f $c $k >> $O/mfma.txt; done
  done
  python3 - "$f" >> $O/mfma.txt <<'EOF'
import csv, collections, sys
dur = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    if ("k_cgemm2" in k or "k_gram" in k) and r.get("Counter_Name") == "SQ_BUSY_CYCLES":
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in dur.items():
    print(f"{k}: duration_us {sum(v) / len(v):.1f} over {len(v)}")
EOF
  find $O/$p -name "*.csv" -delete
done
cat $O/mfma.txt
echo done
