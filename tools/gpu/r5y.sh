#!/bin/bash
# round 5: quad kernel at 2 vs 3 waves/SIMD (launch bounds), interleaved; the box's scratch copy swaps the library
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5y
mkdir -p $O
cd $R
for r in 1 2; do
  for v in qw3 qw2; do
    cp variants/libsv_$v.so stellar-core_amd/libstellar_sigverify.so
    SWEEP_PATHS=quad timeout -k 10 300 python3 tools/size_sweep.py 15 4096,8192,16384,20480,24576,29217,32768 > $O/sweep_${v}_$r.json 2> $O/sweep_${v}_$r.err
  done
done
cp variants/libsv_qw3.so stellar-core_amd/libstellar_sigverify.so
echo done
