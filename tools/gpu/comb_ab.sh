# Warm-key latency A/B of variants/libsv_prev.so vs variants/libsv_prod.so
# (tools/ab_lat_capi.py), then the phase timeline of the current tree
# (tools/comb_phases.py).  Usage: bash tools/gpu/comb_ab.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-comb_ab}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
AB_MODES=${AB_MODES:-warm} AB_ROUNDS=6 AB_ITERS=300 timeout -k 10 400 python -u tools/ab_lat_capi.py $V/libsv_prev.so $V/libsv_prod.so > $OUT/ab_lat.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/comb_phases.py $V/libsv_diag_phases.so > $OUT/phases.txt 2>&1 || exit $?
