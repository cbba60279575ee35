#!/bin/bash
# round 5: config 4 integrated after the harness's main-thread post wakes only a sleeping thread
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5v
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/scp_probe.py 48000 "1000:5000:0:1:2:4,1000:5000:50:1:2:4,1000:5000:0:1:2:4,1000:5000:50:1:2:4,4:200:0:1:2:4" > $O/probe.jsonl 2> $O/probe.err
echo done
