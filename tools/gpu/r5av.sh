#!/bin/bash
# round 5: fail-closed hand-overs in the three-wave octet: octet GPU tests (a dropped hand-over included)
# and the cold latency against the previous kernels (old = this round's commit before it)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5av
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_comb.py tests/test_gpu_parity.py tests/test_gpu_longmsg.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
cp stellar-core_amd/libstellar_sigverify.so /tmp/sv_keep.so
for r in 1 2 3; do
  for v in prev tree; do
    if [ $v = tree ]; then cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
    else cp variants/libsv_$v.so stellar-core_amd/libstellar_sigverify.so; fi
    SV_PROBE_LIB_NAME=$v timeout -k 10 200 python3 tools/cold_probe.py 300 1000,4096 >> $O/cold.jsonl 2>> $O/cold.err
  done
done
cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
echo done
