# A/B: L2 prefetch of the R entry with a counted wait (SV_PFR) against the base
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_pfr}; mkdir -p $OUT
export TMPDIR=/tmp
AB_ROUNDS=${AB_ROUNDS:-12} timeout -k 10 500 python -u tools/ab_variants.py variants/libsv_base.so variants/libsv_pfr.so > $OUT/ab.txt 2>&1
