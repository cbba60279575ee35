#!/bin/bash
# round 5 final evidence: hardware mads per verify (madcount build), then the rocprofv3 kernel trace + PMC passes
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5t
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/madcount.py --out $O/madcount.json > $O/madcount.log 2>&1
bash tools/profile_run.sh $O/prof > $O/profile_run.log 2>&1
echo done
