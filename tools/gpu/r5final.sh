# Round-5 evidence pass on the final tree: GPU suite, smoke, bench (N=1),
# a 2-rank rehearsal of the N>1 line on one GPU (the mad count and the
# rocprofv3 profile of these kernel sources: tools/gpu/r5t.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5final}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
SECONDS=0; timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?; echo "bench wall $SECONDS s" > $OUT/bench_wall.txt
SV_BENCH_SHARE_GPUS=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/bench_n2.json 2> $OUT/bench_n2.err || exit $?
echo done
