#!/bin/bash
# round 5: host-API 2^20 batch with staging chunks of 2^18 (default) / 2^19 / 2^20, interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5al2
mkdir -p $O
cd $R
B="bench.py --steps 6 --warmup 1 --no-cpu --no-latency --no-config1 --no-config4i --no-config35"
for r in 1 2 3; do
  for c in 131072 262144; do
    SV_STAGE_CHUNK=$c timeout -k 10 200 python3 $B > $O/b_${c}_$r.json 2> $O/b_${c}_$r.err
  done
done
echo done
