# Octet kernel with 5-bit windows: 1k latency A/B (warm comb unchanged, cold
# octet) through the C-ABI, product (variants/libsv_prod.so) vs new
# (variants/libsv_oct5.so), then the GPU suite and the octet phase timeline.
# Usage: bash tools/gpu/ab_oct5.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_oct5}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
AB_ROUNDS=6 AB_ITERS=300 timeout -k 10 400 python -u tools/ab_lat_capi.py $V/libsv_prod.so $V/libsv_oct5.so > $OUT/ab_lat.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
