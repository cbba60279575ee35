#!/bin/bash
# round 5 (diagnosis, temporary trace build): where config 3's pair enumeration goes on the box
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ax
mkdir -p $O
cd $R
SV_AB_TRACE=1 timeout -k 10 300 python3 tools/bench_configs.py --configs 3 > $O/config3.json 2> $O/config3.err
echo done
