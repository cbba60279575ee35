# A/B: table-memory variants of the throughput path (nt DMAs, nt stores,
# shared identity entry) against the base
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_mem}; mkdir -p $OUT
export TMPDIR=/tmp
LIBS=$(ls variants/libsv_*.so)
AB_ROUNDS=${AB_ROUNDS:-10} timeout -k 10 500 python -u tools/ab_variants.py $LIBS > $OUT/ab.txt 2>&1
