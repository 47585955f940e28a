#!/bin/bash
# GPU box: the Gram's parity tests, its timings per build (k-steps in flight U = 4 / 8 / 16;
# the diagnostics build's LRS_GRAM_NB / LRS_GRAM_C overrides), then a kernel trace of the
# default build for the k_gram / k_gram_fin split.
set -e
mkdir -p gpurun_out/gram
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k gram -x -q --timeout 120 --timeout-method thread > gpurun_out/gram/tests.log 2>&1
L=ltr-lowrank-sdp_amd/_build
: > gpurun_out/gram/diag.log
for v in liblrsdp liblrsdp_u4 liblrsdp_u16; do
  echo "== $v" >> gpurun_out/gram/diag.log
  LRS_LIB=$L/$v.so timeout -k 10 120 python3 -u scripts/gram_probe.py 100 19,64,128,256,512 >> gpurun_out/gram/diag.log 2>&1
  LRS_LIB=$L/$v.so timeout -k 10 120 python3 -u scripts/gram_probe.py 316 128 >> gpurun_out/gram/diag.log 2>&1
done
for nb in 1 4; do
  echo "== NB=$nb" >> gpurun_out/gram/diag.log
  LRS_GRAM_NB=$nb LRS_LIB=$L/liblrsdp_gd.so timeout -k 10 120 python3 -u scripts/gram_probe.py 100 64,128,256,512 >> gpurun_out/gram/diag.log 2>&1
  LRS_GRAM_NB=$nb LRS_LIB=$L/liblrsdp_gd.so timeout -k 10 120 python3 -u scripts/gram_probe.py 316 128 >> gpurun_out/gram/diag.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gram/prof -o run -- python3 -u $GRAFT_REPO_ROOT/scripts/gram_probe.py 100 19,128 > $GRAFT_REPO_ROOT/gpurun_out/gram/prof.log 2>&1
tail -3 $GRAFT_REPO_ROOT/gpurun_out/gram/tests.log
cat $GRAFT_REPO_ROOT/gpurun_out/gram/diag.log
