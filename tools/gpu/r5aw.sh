#!/bin/bash
# round 5: fail-closed hand-overs: the full version (tree: validity carried through every flag) vs wave 0's
# own waits only (min) vs before (prev), cold latency interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5aw
mkdir -p $O
cd $R
cp stellar-core_amd/libstellar_sigverify.so /tmp/sv_keep.so
for r in 1 2 3 4; do
  for v in prev min tree; do
    if [ $v = tree ]; then cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
    else cp variants/libsv_$v.so stellar-core_amd/libstellar_sigverify.so; fi
    SV_PROBE_LIB_NAME=$v timeout -k 10 200 python3 tools/cold_probe.py 300 1000,3000,4096 >> $O/cold.jsonl 2>> $O/cold.err
  done
done
cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
echo done
