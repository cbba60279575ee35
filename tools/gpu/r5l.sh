#!/bin/bash
# round 5: where a medium host call's time goes (stage trace + kernel trace)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SV_STAGE_TRACE=1 timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe.json 2> $O/probe.err
echo done
