# 2^20 kernel-time A/B: product (3 waves/SIMD main kernel) vs SV_MAIN_WAVES=4
# (tools/build_variants.sh w4 -DSV_MAIN_WAVES=4).  Usage: bash tools/gpu/ab_w4.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_w4}; mkdir -p $OUT
export TMPDIR=/tmp
AB_ROUNDS=10 timeout -k 10 500 python -u tools/ab_variants.py variants/libsv_prod.so variants/libsv_w4.so > $OUT/ab.txt 2>&1 || exit $?
