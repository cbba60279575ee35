# Kernel A/B of variants/libsv_*.so (tools/ab_variants.py), then the GPU suite
# (usage: bash tools/gpu/ab.sh OUTDIR [pytest])
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
export TMPDIR=/tmp
AB_ROUNDS=${AB_ROUNDS:-8} timeout -k 10 600 python -u tools/ab_variants.py $AB_LIBS > $OUT/ab.txt 2>&1 || exit $?
if [ "$2" = pytest ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
fi
