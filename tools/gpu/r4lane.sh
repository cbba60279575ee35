# Evidence pass after a host-side (sv_api.cpp) change: GPU suite, smoke, bench
# (N=1), the 2-rank rehearsal, and the isolation run.  Kernel sources are
# unchanged, so the mad count and the rocprofv3 profile keyed to their digest
# stand.  Usage: bash tools/gpu/r4lane.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4lane}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
SV_BENCH_SHARE_GPUS=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/bench_n2.json 2> $OUT/bench_n2.err || exit $?
SV_ISOLATION_OUT=$OUT/isolation_shared.json timeout -k 10 300 python -u -m pytest tests/test_gpu_isolation.py -x -q -s --timeout 240 --timeout-method thread > $OUT/iso.txt 2>&1 || exit $?
