# Integration-layer timings on the GPU box (tools/host_bench.cpp, built in-tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-hb1}; mkdir -p $OUT
SV_HOST_TRACE=1 timeout -k 10 300 ./tools/host_bench 100000 gpu > $OUT/host_bench.txt 2> $OUT/trace.txt
