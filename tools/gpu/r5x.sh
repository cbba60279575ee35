#!/bin/bash
# round 5: config 3 with the tx objects kept per thread (three runs)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5x
mkdir -p $O
cd $R
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/txset_host_probe.py 5000 2 10 > $O/probe_$r.txt 2>&1
  timeout -k 10 300 python3 tools/bench_configs.py --configs 3 > $O/config3_$r.json 2> $O/config3_$r.err
done
echo done
