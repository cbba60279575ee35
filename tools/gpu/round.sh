# Full GPU check: parity suite, mad count (when the measurement build exists), bench
# (usage: bash tools/gpu/round.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-round1}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
if [ -f variants/libsv_madcount.so ]; then
  timeout -k 10 300 python -u tools/madcount.py --out $OUT/madcount.json > $OUT/madcount.txt 2>&1 || exit $?
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
