#!/bin/bash
# round 5: three-wave cold octet at the default threshold (4096) -- GPU suite, cold-key latency old / new
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ai
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for r in 1 2; do
  cp variants/libsv_oldoct.so stellar-core_amd/libstellar_sigverify.so
  SV_PROBE_LIB_NAME=old timeout -k 10 200 python3 tools/cold_probe.py 300 1000,2048,4096,5000,6144 >> $O/cold.jsonl 2>> $O/cold.err
  cp variants/libsv_newoct.so stellar-core_amd/libstellar_sigverify.so
  SV_PROBE_LIB_NAME=new timeout -k 10 200 python3 tools/cold_probe.py 300 1000,2048,4096,5000,6144 >> $O/cold.jsonl 2>> $O/cold.err
done
echo done
