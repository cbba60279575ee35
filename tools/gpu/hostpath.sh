# Host-integration GPU tests + verifySigBatch timings (usage: bash tools/gpu/hostpath.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-hp1}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_host_mirror.py tests/test_wrapper.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || exit $?
SV_HOST_TRACE=1 timeout -k 10 180 ./tools/host_bench 100000 gpu > $OUT/host_bench.txt 2> $OUT/trace.txt
