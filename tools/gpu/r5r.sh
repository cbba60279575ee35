#!/bin/bash
# round 5: in-place verdicts for one-chunk batches -- full GPU suite, then sweep / probe with and without
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5r
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for z in 1 0; do
  SV_BULK_ZC_OUT=$z SWEEP_PATHS=auto timeout -k 10 300 python3 tools/size_sweep.py 15 12289,16384,24576,29217,32768,50000,100000,131072 > $O/sweep_zo$z.json 2> $O/sweep_zo$z.err
done
for z in 1 0; do
  SV_BULK_ZC_OUT=$z SWEEP_PATHS=auto timeout -k 10 300 python3 tools/size_sweep.py 15 12289,16384,24576,29217,32768,50000,100000,131072 > $O/sweep2_zo$z.json 2> $O/sweep2_zo$z.err
done
echo done
