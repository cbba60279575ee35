#!/bin/bash
# round 5: one-chunk staging A/B (pipelined sections / one copy / in place), kernel trace + stage trace
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in pipe:SV_PIPELINED_PACK=1 one:SV_PIPELINED_PACK=0 zc:SV_BULK_ZC_IN=1; do
  name=${v%%:*}; kv=${v#*:}
  export ${kv}
  SV_STAGE_TRACE=1 timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt_$name -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,50000,100000 > $O/probe_$name.json 2> $O/probe_$name.err
  unset ${kv%%=*}
done
for v in pipe:SV_PIPELINED_PACK=1 zc:SV_BULK_ZC_IN=1; do
  name=${v%%:*}; kv=${v#*:}
  export ${kv}
  SWEEP_PATHS=auto timeout -k 10 300 python3 $R/tools/size_sweep.py 15 4096,8192,16384,24576,29217,32768,50000,100000,131072 > $O/sweep_$name.json 2> $O/sweep_$name.err
  unset ${kv%%=*}
done
echo done
