# Isolation run, twice, recording the engine's own time per latency batch
# beside the Python wall time.  Usage: bash tools/gpu/iso_eng.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-iso_eng}; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  SV_ISOLATION_OUT=$OUT/isolation_$r.json timeout -k 10 300 python -u -m pytest tests/test_gpu_isolation.py -x -q -s --timeout 240 --timeout-method thread > $OUT/iso_$r.txt 2>&1 || exit $?
done
