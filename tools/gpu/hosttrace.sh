# verifySigBatch keyed 100k with engine stage tracing (usage: bash tools/gpu/hosttrace.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ht1}; mkdir -p $OUT
SV_STAGE_TRACE=1 SV_HOST_TRACE=1 timeout -k 10 180 ./tools/host_bench 100000 gpu > $OUT/host_bench.txt 2> $OUT/trace.txt
