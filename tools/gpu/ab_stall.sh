# Where the main kernel waits: A/B of base / A-R-table alias / base-table alias
# (diagnostic builds, wrong verdicts by design), then one SQ stall-counter
# pass per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_stall}; mkdir -p $OUT
export TMPDIR=/tmp
V="base alias64 btalias"
LIBS=""; for v in $V; do LIBS="$LIBS variants/libsv_$v.so"; done
AB_NOCHECK=alias AB_ROUNDS=${AB_ROUNDS:-10} timeout -k 10 400 python -u tools/ab_variants.py $LIBS > $OUT/ab.txt 2>&1 || exit $?
cd /tmp
for v in $V; do
  AB_NOCHECK=alias AB_ROUNDS=4 timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/$OUT/sq_$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/ab_variants.py $GRAFT_REPO_ROOT/variants/libsv_$v.so > $GRAFT_REPO_ROOT/$OUT/sq_$v.log 2>&1 || exit $?
done
