#!/bin/bash
# round 5: two latency-lane contexts -- GPU suite, then config 4 with 1 / 2 contexts and 1 / 2 batches in flight
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5w
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
G="1000:5000:0:1:2:4,1000:5000:0:2:2:4,1000:5000:30:2:2:4,1000:5000:0:1:2:4,1000:5000:0:2:2:4,1000:5000:30:2:2:4,4:200:0:2:2:4"
for c in 2 1; do
  SV_LAT_CONTEXTS=$c timeout -k 10 300 python3 tools/scp_probe.py 48000 "$G" > $O/probe_ctx$c.jsonl 2> $O/probe_ctx$c.err
done
echo done
