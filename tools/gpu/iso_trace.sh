# Isolation run with the latency lane's per-batch stage trace (SV_LAT_TRACE)
# to find where 1k batches wait while the 2^22 host batch runs.
# Usage: bash tools/gpu/iso_trace.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-iso_trace}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$STAGE" ]; then export SV_STAGE_TRACE=1; fi  # (the bulk calls' stages too)
SV_LAT_TRACE=1 SV_ISOLATION_OUT=$OUT/isolation_shared.json timeout -k 10 300 python -u -m pytest tests/test_gpu_isolation.py -x -q -s --timeout 240 --timeout-method thread > $OUT/iso.txt 2> $OUT/trace.txt || exit $?
