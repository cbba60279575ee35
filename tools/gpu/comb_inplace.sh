# Comb / octet phase timelines with the lane's input read in place, and the
# product vs the no-SHA diagnostic build (what the hash, loads included, costs).
# Usage: bash tools/gpu/comb_inplace.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-comb_inplace}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
timeout -k 10 120 python -u tools/comb_phases.py $V/libsv_diag_phases.so > $OUT/phases.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/comb_phases.py --octet $V/libsv_diag_ophases.so > $OUT/ophases.txt 2>&1 || exit $?
SV_LAT_ZC_IN=0 timeout -k 10 120 python -u tools/comb_phases.py $V/libsv_diag_phases.so > $OUT/phases_staged.txt 2>&1 || exit $?
AB_MODES=warm AB_ROUNDS=4 AB_ITERS=300 timeout -k 10 400 python -u tools/ab_lat_capi.py stellar-core_amd/libstellar_sigverify.so \
    $V/libsv_diag_nohash.so $V/libsv_diag_nodecode.so > $OUT/ab_lat.txt 2>&1 || exit $?
