# A/B of the verifySigBatch cache walk: variants/hostold (previous libstellar_host.so)
# vs the in-tree one, stub engine and GPU engine, interleaved (usage: bash tools/gpu/hostwalk_ab.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-hwab}; mkdir -p $OUT
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export LD_LIBRARY_PATH=$PWD/variants/hostold:$PWD/stellar-core_amd; else unset LD_LIBRARY_PATH; fi
    SV_HOST_TRACE=1 SV_STAGE_TRACE=1 timeout -k 10 120 ./tools/host_bench 100000 gpu > $OUT/hb_${v}_$r.txt 2> $OUT/trace_${v}_$r.txt || exit $?
  done
done
