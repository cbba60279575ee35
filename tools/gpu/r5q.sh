#!/bin/bash
# round 5: gate nap / publication-piece variants (the box's scratch copy swaps the library per variant)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in nap16 nap4 nap1; do
  cp $R/variants/libsv_$v.so $R/stellar-core_amd/libstellar_sigverify.so
  for pc in 1024 4096; do
    SV_GATE_PIECE=$pc timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt_${v}_$pc -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,100000 > $O/probe_${v}_$pc.json 2> $O/probe_${v}_$pc.err
  done
done
cp $R/variants/libsv_nap16.so $R/stellar-core_amd/libstellar_sigverify.so
SV_GATED=0 timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace -d $O/kt_nogate -o kt -- python3 $R/tools/host_call_probe.py 6 16384,29217,100000 > $O/probe_nogate.json 2> $O/probe_nogate.err
echo done
