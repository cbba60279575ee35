# Round 5: message windows staged with every load in flight at once (comb /
# octet / quad kernels): GPU suite, bench, the auto column at latency sizes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
SWEEP_PATHS=auto timeout -k 10 400 python -u tools/size_sweep.py 15 "1000,2048,4096,6144,8192,12288,16384,29217,32768" > $OUT/size_sweep.json 2> $OUT/size_sweep.err || exit $?
