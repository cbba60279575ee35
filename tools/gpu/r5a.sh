# Round-5 first pass: GPU suite (new: config-4 integrated path, staged keyed /
# bulk fallbacks), the medium-size sweep of both kernel paths, the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5a}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/size_sweep.py 15 > $OUT/size_sweep.json 2> $OUT/size_sweep.err || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
