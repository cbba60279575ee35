# HIP API round-trip probe + traced latency-lane batches (usage: bash tools/gpu/lat_api.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-api1}; mkdir -p $OUT
timeout -k 10 120 ./tools/gpu/api_probe.bin > $OUT/api_probe.txt 2>&1 || exit $?
SV_LAT_TRACE=1 timeout -k 10 300 python tools/lat_probe.py --sizes 1000 --iters 30 --cold 0 > $OUT/probe.txt 2> $OUT/trace.txt
