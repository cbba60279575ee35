#!/bin/bash
# round 5: one-chunk host batches read in place (default) vs staged (SV_BULK_ZC_IN=0) with the
# 256 KB pack tasks, interleaved, plus the per-stage trace of one call each
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5at
mkdir -p $O
cd $R
for r in 1 2 3; do
  for z in 1 0; do
    SV_BULK_ZC_IN=$z timeout -k 10 200 python3 tools/size_sweep.py 15 16384,29217,50000 > $O/sweep_zc${z}_$r.json 2> $O/sweep_zc${z}_$r.err
  done
done
for z in 1 0; do
  SV_BULK_ZC_IN=$z SV_STAGE_TRACE=1 timeout -k 10 200 python3 tools/host_call_probe.py 6 29217 > $O/probe_zc$z.txt 2>&1
done
echo done
