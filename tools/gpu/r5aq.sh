#!/bin/bash
# round 5: config 4 tails on the final tree (paced and trickle, three repeats each), after the
# 1.7 ms p99 of bench_r5final4 (one run)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5aq
mkdir -p $O
cd $R
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/scp_probe.py 12000 "1000:5000:0:1:2:4,4:200:0:1:2:4,1000:5000:0:1:2:4,4:200:0:1:2:4" \
      >> $O/probe.jsonl 2>> $O/probe.err
done
echo done
