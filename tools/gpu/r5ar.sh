#!/bin/bash
# round 5: bytes per pack task (SV_PACK_PART: 1 MB = 3 tasks for a 29k batch; 256 KB / 128 KB use the
# whole pool), interleaved: medium host calls (size sweep) and cold 1k lane calls
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ar
mkdir -p $O
cd $R
for r in 1 2 3; do
  for p in 1048576 262144 131072; do
    SV_PACK_PART=$p timeout -k 10 200 python3 tools/size_sweep.py 15 8192,16384,29217,50000,100000 > $O/sweep_${p}_$r.json 2> $O/sweep_${p}_$r.err
    SV_PACK_PART=$p SV_PROBE_LIB_NAME=p$p timeout -k 10 200 python3 tools/cold_probe.py 300 1000 >> $O/cold.jsonl 2>> $O/cold.err
  done
done
echo done
