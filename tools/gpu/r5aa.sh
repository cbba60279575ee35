#!/bin/bash
# round 5: config 3 (variable-length messages) with the one-chunk image staged vs read in place, interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5aa
mkdir -p $O
cd $R
for r in 1 2 3; do
  for z in 1 0; do
    SV_BULK_ZC_IN=$z timeout -k 10 300 python3 tools/bench_configs.py --configs 3 > $O/config3_zc${z}_$r.json 2> $O/config3_zc${z}_$r.err
  done
done
echo done
