# Integration-layer checks on the GPU box: config-3 phase trace, host bench
# (verifySigBatch / tx set / micro-batcher), GPU tests of the host mirror and wrapper
# (usage: bash tools/gpu/host_round.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-hr}; mkdir -p $OUT
export TMPDIR=/tmp
SV_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_configs.py --configs 3 > $OUT/c3.json 2> $OUT/c3.err || exit $?
SV_HOST_TRACE=1 timeout -k 10 300 ./tools/host_bench 100000 gpu > $OUT/host_bench.txt 2> $OUT/trace.txt || exit $?
timeout -k 10 600 python -u -m pytest tests/test_host_mirror.py tests/test_wrapper.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu_host.txt 2>&1
