#!/bin/bash
# round 5: three-wave octet with LDS-flag hand-overs (the high wave starts at the decoded points):
# octet GPU tests, then cold latency interleaved against the barrier version (old) and split divisors
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5an
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_comb.py tests/test_gpu_parity.py tests/test_gpu_longmsg.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
cp stellar-core_amd/libstellar_sigverify.so /tmp/sv_keep.so
for r in 1 2 3; do
  for v in old d4 d5 d6 d7; do
    cp variants/libsv_$v.so stellar-core_amd/libstellar_sigverify.so
    SV_PROBE_LIB_NAME=$v timeout -k 10 200 python3 tools/cold_probe.py 300 1000,2048,4096 >> $O/cold.jsonl 2>> $O/cold.err
  done
done
cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
echo done
