#!/bin/bash
# round 5: three-wave octet split point (SV_OCT_HI_DIV: the high wave takes about W / DIV windows), interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ak
mkdir -p $O
cd $R
cp stellar-core_amd/libstellar_sigverify.so /tmp/sv_keep.so
for r in 1 2 3; do
  for v in d6 d7 d9 d11 d14; do
    cp variants/libsv_$v.so stellar-core_amd/libstellar_sigverify.so
    SV_PROBE_LIB_NAME=$v timeout -k 10 200 python3 tools/cold_probe.py 300 1000,2048,4096 >> $O/cold.jsonl 2>> $O/cold.err
  done
done
cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
echo done
