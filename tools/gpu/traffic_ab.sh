# Diagnostic A/B: what the main kernel's beyond-L2 table traffic costs.
# Variants (tools/build_variants.sh): base, alias64 (main reads every wave's
# tables from one 64-signature region: L2-resident), alias64k (a 65,536-
# signature region, ~189 MB: Infinity-Cache-resident), alias64both (prep
# writes aliased too).  Verdicts of the alias builds are wrong by design.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-traffic_ab}; mkdir -p $OUT
export TMPDIR=/tmp
V="base alias64 alias64k alias64both"
LIBS=""; for v in $V; do LIBS="$LIBS variants/libsv_$v.so"; done
AB_NOCHECK=alias AB_ROUNDS=${AB_ROUNDS:-8} timeout -k 10 400 python -u tools/ab_variants.py $LIBS > $OUT/ab.txt 2>&1 || exit $?
cd /tmp
for v in $V; do
  AB_NOCHECK=alias AB_ROUNDS=3 timeout -k 10 120 rocprofv3 --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU -d $GRAFT_REPO_ROOT/$OUT/clk_$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/ab_variants.py $GRAFT_REPO_ROOT/variants/libsv_$v.so > $GRAFT_REPO_ROOT/$OUT/clk_$v.log 2>&1 || exit $?
  AB_NOCHECK=alias AB_ROUNDS=3 timeout -k 10 120 rocprofv3 --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum -d $GRAFT_REPO_ROOT/$OUT/l2_$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/ab_variants.py $GRAFT_REPO_ROOT/variants/libsv_$v.so > $GRAFT_REPO_ROOT/$OUT/l2_$v.log 2>&1 || exit $?
done
