# verifySigBatch cache-walk cost vs batch size on the GPU box (tools/host_bench.cpp)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-hw1}; mkdir -p $OUT
for n in 30000 60000 100000 200000; do
  SV_HOST_TRACE=1 timeout -k 10 120 ./tools/host_bench $n > $OUT/hb_$n.txt 2> $OUT/trace_$n.txt || exit $?
done
