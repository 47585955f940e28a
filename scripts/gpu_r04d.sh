#!/bin/bash
# Round 4: the headline (G67 ALM it/s) with and without the latency kernels' prefetch records
# (LRS_LAT_REC), their bit-identity test, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04d; mkdir -p $O
H="--no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --no-sharded"
for v in 1 0 1 0; do
  LRS_LAT_REC=$v timeout -k 10 200 python3 -u bench.py --steps 3000 --warmup 300 $H > $O/head_$v.log 2>&1 || { tail -5 $O/head_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('LRS_LAT_REC=$v', d['value'], d['ms_per_step'], d['roofline'])" $O/head_$v.log | tee -a $O/head.txt
done
timeout -k 10 300 python3 -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_bundled.py -k lat_prefetch > $O/pytest_rec.txt 2>&1 || { tail -20 $O/pytest_rec.txt; exit 1; }
tail -3 $O/pytest_rec.txt
timeout -k 10 800 python3 -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.txt | head -20
tail -3 $O/pytest.txt
exit $rc
