#!/bin/bash
# round 5: the size-dependent pack task (1 MB below 2 MB packs, 256 KB above): medium host-call tests and
# a size sweep against the all-1 MB setting, interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5as
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_medium_host.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.txt 2>&1
for r in 1 2 3; do
  for p in 1048576 tree; do
    if [ $p = tree ]; then env -u SV_PACK_PART timeout -k 10 200 python3 tools/size_sweep.py 15 8192,16384,29217,50000 > $O/sweep_${p}_$r.json 2> $O/sweep_${p}_$r.err
    else SV_PACK_PART=$p timeout -k 10 200 python3 tools/size_sweep.py 15 8192,16384,29217,50000 > $O/sweep_${p}_$r.json 2> $O/sweep_${p}_$r.err; fi
  done
done
echo done
