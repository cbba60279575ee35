# Isolation evidence on the final tree: 1k latency batches under a 2^22 host
# batch and a 2^24 device batch (tests/test_gpu_isolation.py), stats to
# SV_ISOLATION_OUT.  Usage: bash tools/gpu/iso_r4.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-iso_r4}; mkdir -p $OUT
export TMPDIR=/tmp
SV_ISOLATION_OUT=$OUT/isolation_shared.json timeout -k 10 300 python -u -m pytest tests/test_gpu_isolation.py -x -q -s --timeout 240 --timeout-method thread > $OUT/iso.txt 2>&1 || exit $?
