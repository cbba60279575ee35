# Round-4 GPU pass: full GPU suite, kernel A/B (bitop3 SHA, table-traffic
# diagnostics), the bench, PMC clock / L2 passes of the A/B variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4b}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
V="base prevsha alias64 alias64k alias64both"
LIBS=""; for v in $V; do LIBS="$LIBS variants/libsv_$v.so"; done
AB_NOCHECK=alias AB_ROUNDS=${AB_ROUNDS:-8} timeout -k 10 400 python -u tools/ab_variants.py $LIBS > $OUT/ab.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cd /tmp
for v in base alias64 alias64k; do
  AB_NOCHECK=alias AB_ROUNDS=3 timeout -k 10 120 rocprofv3 --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU -d $GRAFT_REPO_ROOT/$OUT/clk_$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/ab_variants.py $GRAFT_REPO_ROOT/variants/libsv_$v.so > $GRAFT_REPO_ROOT/$OUT/clk_$v.log 2>&1 || exit $?
  AB_NOCHECK=alias AB_ROUNDS=3 timeout -k 10 120 rocprofv3 --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum -d $GRAFT_REPO_ROOT/$OUT/l2_$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/ab_variants.py $GRAFT_REPO_ROOT/variants/libsv_$v.so > $GRAFT_REPO_ROOT/$OUT/l2_$v.log 2>&1 || exit $?
done
