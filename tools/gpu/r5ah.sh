#!/bin/bash
# round 5: three-wave cold octet kernel -- GPU suite, then cold-key latency: old kernels / new with the third
# wave off / on, interleaved (the box's scratch copy swaps the library)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ah
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for r in 1 2 3; do
  cp variants/libsv_oldoct.so stellar-core_amd/libstellar_sigverify.so
  SV_PROBE_LIB_NAME=old timeout -k 10 200 python3 tools/cold_probe.py 300 1000,2048,4096,6144 >> $O/cold.jsonl 2>> $O/cold.err
  cp variants/libsv_newoct.so stellar-core_amd/libstellar_sigverify.so
  SV_PROBE_LIB_NAME=new SV_OCT_HI_MAX=0 timeout -k 10 200 python3 tools/cold_probe.py 300 1000,2048,4096,6144 >> $O/cold.jsonl 2>> $O/cold.err
  SV_PROBE_LIB_NAME=new SV_OCT_HI_MAX=100000 timeout -k 10 200 python3 tools/cold_probe.py 300 1000,2048,4096,6144 >> $O/cold.jsonl 2>> $O/cold.err
done
cp variants/libsv_newoct.so stellar-core_amd/libstellar_sigverify.so
echo done
