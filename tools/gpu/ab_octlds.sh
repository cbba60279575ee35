# Cold-key octet kernel: product vs its tables in dynamic LDS (v1dyn) vs 5-bit
# windows with dynamic LDS (v2oct5), 1k cold p50 through the C-ABI.
# Usage: bash tools/gpu/ab_octlds.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_octlds}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
AB_MODES=cold AB_ROUNDS=8 AB_ITERS=300 timeout -k 10 400 python -u tools/ab_lat_capi.py $V/libsv_prod.so $V/libsv_v1dyn.so $V/libsv_v2oct5.so > $OUT/ab_lat.txt 2>&1 || exit $?
