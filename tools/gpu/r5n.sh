#!/bin/bash
# round 5: H2D copy rate by size / streams, SDMA vs shader copies
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5n
mkdir -p $O
timeout -k 10 120 python3 $R/tools/h2d_probe.py > $O/h2d_sdma.json 2> $O/h2d_sdma.err
HSA_ENABLE_SDMA=0 timeout -k 10 120 python3 $R/tools/h2d_probe.py > $O/h2d_blit.json 2> $O/h2d_blit.err
HSA_ENABLE_SDMA=0 timeout -k 10 240 python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe_blit.json 2> $O/probe_blit.err
timeout -k 10 240 python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe_sdma.json 2> $O/probe_sdma.err
echo done
