# Round 5: product-form A/B (generated asm statements vs the column-major C++
# forms on the device) on the bench kernels, interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5g}; mkdir -p $OUT
export TMPDIR=/tmp
AB_ROUNDS=8 timeout -k 10 400 python -u tools/ab_variants.py variants/libsv_base.so variants/libsv_cm.so > $OUT/ab_cm.txt 2>&1 || exit $?
