# Round 5: one-chunk host batches read in place vs staged (SV_BULK_ZC_IN) on
# the quad geometry, per call and through config 3; interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5k}; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for z in 1 0; do
SV_BULK_ZC_IN=$z SWEEP_PATHS=auto timeout -k 10 300 python -u tools/size_sweep.py 15 "16384,24576,29217,32768,50000,100000" > $OUT/sweep_zc${z}_$r.json 2> $OUT/sweep_zc${z}_$r.err || exit $?
SV_BULK_ZC_IN=$z timeout -k 10 300 python -u tools/bench_configs.py --configs 3 > $OUT/config3_zc${z}_$r.json 2> $OUT/config3_zc${z}_$r.err || exit $?
done
done
