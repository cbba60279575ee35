#!/bin/bash
# round 5: gate poll variants (SV_GATE_MODE 0 relaxed + one acquire, 1 acquire per poll, 2 relaxed only)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5p
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gated.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gated.txt 2>&1
cd /tmp && export TMPDIR=/tmp
for g in 0 1 2; do
SV_GATE_MODE=$g timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt_m$g -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe_m$g.json 2> $O/probe_m$g.err
done
SV_GATED=0 timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt_nogate -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe_nogate.json 2> $O/probe_nogate.err
echo done
