# Where the warm-key comb kernel's time goes: product vs diagnostic builds
# (tools/build_comb_diag.sh) through tools/ab_lat_capi.py, warm keys only.
# Usage: bash tools/gpu/comb_diag.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-comb_diag}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
AB_MODES=warm AB_ROUNDS=4 AB_ITERS=300 timeout -k 10 400 python -u tools/ab_lat_capi.py $V/libsv_prod.so \
    $V/libsv_diag_nodecode.so $V/libsv_diag_nohash.so $V/libsv_diag_both.so > $OUT/ab_lat.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/comb_phases.py $V/libsv_diag_phases.so > $OUT/phases.txt 2>&1 || exit $?
