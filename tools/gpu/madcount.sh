# Hardware mad count per verify (variants/libsv_madcount.so built by tools/build_variants.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-mc1}; mkdir -p $OUT
timeout -k 10 300 python -u tools/madcount.py --out $OUT/madcount.json > $OUT/madcount.txt 2>&1
