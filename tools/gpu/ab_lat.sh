# Lattice-reduction rewrite A/B: 1k latency (warm comb / cold octet) through
# the C-ABI and 2^20 kernel time, product (variants/libsv_prod.so) vs new
# (variants/libsv_lat.so), then the GPU suite on the new tree.
# Usage: bash tools/gpu/ab_lat.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_lat}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
AB_ROUNDS=6 AB_ITERS=300 timeout -k 10 400 python -u tools/ab_lat_capi.py $V/libsv_prod.so $V/libsv_lat.so > $OUT/ab_lat.txt 2>&1 || exit $?
AB_ROUNDS=8 timeout -k 10 400 python -u tools/ab_variants.py $V/libsv_prod.so $V/libsv_lat.so > $OUT/ab_tp.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
