# A/B: L2 prefetch of the late-staged table entries (SV_PF) against the base
# and the all-L2 diagnostic bound (alias64)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_pf}; mkdir -p $OUT
export TMPDIR=/tmp
LIBS="variants/libsv_base.so variants/libsv_pf1.so variants/libsv_pf2.so variants/libsv_pf3.so variants/libsv_alias64.so"
AB_NOCHECK=alias AB_ROUNDS=${AB_ROUNDS:-10} timeout -k 10 500 python -u tools/ab_variants.py $LIBS > $OUT/ab.txt 2>&1
