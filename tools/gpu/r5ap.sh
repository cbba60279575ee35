#!/bin/bash
# round 5: (1) GPU tests on the tree; (2) own-form DPP moves with bound_ctrl (tree) vs without (nobc): cold
# latency and the quad kernel's sizes, interleaved; (3) tx-set pre-pass with dynamic parts and a per-tx
# enumerate (tree host library) vs the previous host library (old), interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ap
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_comb.py tests/test_gpu_parity.py tests/test_gpu_longmsg.py \
    tests/test_gpu_medium_host.py tests/test_host_mirror.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
cp stellar-core_amd/libstellar_sigverify.so /tmp/sv_keep.so
cp stellar-core_amd/libstellar_host.so /tmp/svh_keep.so
for r in 1 2 3; do
  for v in nobc tree; do
    if [ $v = tree ]; then cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
    else cp variants/libsv_$v.so stellar-core_amd/libstellar_sigverify.so; fi
    SV_PROBE_LIB_NAME=$v timeout -k 10 200 python3 tools/cold_probe.py 300 1000,4096 >> $O/cold.jsonl 2>> $O/cold.err
    timeout -k 10 200 python3 tools/size_sweep.py 15 16384,29217 > $O/sweep_${v}_$r.json 2> $O/sweep_${v}_$r.err
  done
done
cp /tmp/sv_keep.so stellar-core_amd/libstellar_sigverify.so
for r in 1 2 3; do
  for v in old tree; do
    if [ $v = tree ]; then cp /tmp/svh_keep.so stellar-core_amd/libstellar_host.so
    else cp variants/libstellar_host_old.so stellar-core_amd/libstellar_host.so; fi
    timeout -k 10 200 python3 tools/txset_host_probe.py 5000 2 10 > $O/probe_${v}_$r.txt 2>&1
    timeout -k 10 300 python3 tools/bench_configs.py --configs 3 > $O/config3_${v}_$r.json 2> $O/config3_${v}_$r.err
  done
done
cp /tmp/svh_keep.so stellar-core_amd/libstellar_host.so
echo done
