#!/bin/bash
# round 5: gated one-chunk launches -- parity tests, then the host-call timeline gated / ungated
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5o
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gated.py -x -v --timeout 120 --timeout-method thread > $O/pytest_gated.txt 2>&1
cd /tmp && export TMPDIR=/tmp
SV_STAGE_TRACE=1 timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt_gate -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe_gate.json 2> $O/probe_gate.err
SV_GATED=0 SV_STAGE_TRACE=1 timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt_nogate -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe_nogate.json 2> $O/probe_nogate.err
SWEEP_PATHS=auto timeout -k 10 300 python3 $R/tools/size_sweep.py 15 4096,8192,12289,16384,24576,29217,32768,50000,100000,131072 > $O/sweep_gate.json 2> $O/sweep_gate.err
SV_GATED=0 SWEEP_PATHS=auto timeout -k 10 300 python3 $R/tools/size_sweep.py 15 4096,8192,12289,16384,24576,29217,32768,50000,100000,131072 > $O/sweep_nogate.json 2> $O/sweep_nogate.err
echo done
