#!/bin/bash
# round 5: config 3 host phases, the fused marshal + pair enumeration (new) vs the previous host library (base),
# interleaved; the box's scratch copy swaps libstellar_host.so per run
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5s
mkdir -p $O
cd $R
for r in 1 2 3; do
  for v in base new; do
    cp variants/libstellar_host_$v.so stellar-core_amd/libstellar_host.so
    timeout -k 10 200 python3 tools/txset_host_probe.py 5000 2 10 > $O/probe_${v}_$r.txt 2>&1
    timeout -k 10 300 python3 tools/bench_configs.py --configs 3 > $O/config3_${v}_$r.json 2> $O/config3_${v}_$r.err
  done
done
cp variants/libstellar_host_new.so stellar-core_amd/libstellar_host.so
echo done
