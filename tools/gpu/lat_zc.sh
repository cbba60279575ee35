# zero-copy vs staged latency batches + comb parity (usage: bash tools/gpu/lat_zc.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-zc1}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_comb.py -x -v --timeout 150 --timeout-method thread > $OUT/pytest.txt 2>&1 || exit $?
SV_LAT_ZERO_COPY=0 timeout -k 10 300 python tools/lat_probe.py --sizes 1000,2048,4096 --iters 50 > $OUT/probe_staged.txt 2>&1 || exit $?
SV_LAT_ZERO_COPY=1 timeout -k 10 300 python tools/lat_probe.py --sizes 1000,2048,4096 --iters 50 > $OUT/probe_zc.txt 2>&1
