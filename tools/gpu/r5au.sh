#!/bin/bash
# round 5: does the three-wave octet (hand-overs, W/4 split) now pay above 4096 cold signatures?
# SV_OCT_HI_MAX 4096 (default) vs 6144, interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5au
mkdir -p $O
cd $R
for r in 1 2 3; do
  for m in 4096 6144; do
    SV_OCT_HI_MAX=$m SV_PROBE_LIB_NAME=max$m timeout -k 10 200 python3 tools/cold_probe.py 200 4096,5120,6144 >> $O/cold.jsonl 2>> $O/cold.err
  done
done
echo done
