# Timing experiment: the comb kernel without R's square root (variants/libsv_nodecode.so, wrong
# verdicts) vs the product, latency_1k only (usage: bash tools/gpu/nodecode.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-nd}; mkdir -p $OUT
export TMPDIR=/tmp
B="--steps 2 --warmup 1 --no-cpu --no-host-api --no-config1 --no-config35"
timeout -k 10 300 python -u bench.py $B > $OUT/bench_product.json 2> $OUT/product.err || exit $?
cp stellar-core_amd/libstellar_sigverify.so $OUT/.prod.so
cp variants/libsv_nodecode.so stellar-core_amd/libstellar_sigverify.so
timeout -k 10 300 python -u bench.py $B > $OUT/bench_nodecode.json 2> $OUT/nodecode.err; rc=$?
cp $OUT/.prod.so stellar-core_amd/libstellar_sigverify.so; rm -f $OUT/.prod.so
exit $rc
