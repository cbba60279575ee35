#!/bin/bash
# round 5: keyed micro-batcher batches with the cache keys hashed on the host pool beside a verdicts-only
# engine call (SV_HOST_KEYS=1) vs the engine hash kernel (0, the default): host-mirror GPU tests, then
# config 4 (paced, trickle) interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5az
mkdir -p $O
cd $R
SV_HOST_KEYS=1 timeout -k 10 400 python3 -u -m pytest tests/test_host_mirror.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.txt 2>&1
for r in 1 2 3; do
  for k in 0 1; do
    SV_HOST_KEYS=$k timeout -k 10 200 python3 tools/scp_probe.py 12000 "1000:5000:0:1:2:4,4:200:0:1:2:4,1000:5000:0:1:2:4" \
        > $O/probe_k${k}_$r.jsonl 2> $O/probe_k${k}_$r.err
  done
done
echo done
