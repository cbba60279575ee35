#!/bin/bash
# round 5: quad kernel, A and R loaded first and decoded before S, the message and the hash (tree) vs
# before (prev): quad GPU tests, then medium sizes (kernel and host call), interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ba
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_medium_host.py tests/test_gpu_engine.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
cp stellar-core_amd/libstellar_sigverify.so /tmp/sv_keep.so
for r in 1 2 3; do
  for v in prev tree; do
    if [ $v = tree ]; then cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
    else cp variants/libsv_$v.so stellar-core_amd/libstellar_sigverify.so; fi
    timeout -k 10 200 python3 tools/size_sweep.py 15 12288,16384,29217 > $O/sweep_${v}_$r.json 2> $O/sweep_${v}_$r.err
  done
done
cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
echo done
