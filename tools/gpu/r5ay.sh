#!/bin/bash
# round 5: tx-set pre-pass with the signer payload held inline and parts claimed dynamically (tree) vs the
# previous host library (old): config 3 (distinct sets), interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ay
mkdir -p $O
cd $R
cp stellar-core_amd/libstellar_host.so /tmp/svh_keep.so
for r in 1 2 3 4; do
  for v in old tree; do
    if [ $v = tree ]; then cp /tmp/svh_keep.so stellar-core_amd/libstellar_host.so
    else cp variants/libstellar_host_old.so stellar-core_amd/libstellar_host.so; fi
    timeout -k 10 300 python3 tools/bench_configs.py --configs 3 > $O/config3_${v}_$r.json 2> $O/config3_${v}_$r.err
  done
done
cp /tmp/svh_keep.so stellar-core_amd/libstellar_host.so
echo done
