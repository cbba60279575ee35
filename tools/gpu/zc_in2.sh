# In-place latency input, second pass: SCP-shaped batches of 1000 / 4096 /
# 12288 signatures staged (SV_LAT_ZC_IN=0) vs always in place (2), twice
# alternating, then the isolation run with in place always.
# Usage: bash tools/gpu/zc_in2.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-zc_in2}; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for m in 0 2; do
    SV_LAT_ZC_IN=$m timeout -k 10 200 python -u tools/lat_probe.py --sizes 1000,4096,12288 --iters 200 --out $OUT/probe_m${m}_r${r}.json > $OUT/probe_m${m}_r${r}.txt 2>&1 || exit $?
  done
done
SV_LAT_ZC_IN=2 SV_STAGE_TRACE=1 SV_LAT_TRACE=1 SV_ISOLATION_OUT=$OUT/isolation_shared.json timeout -k 10 300 python -u -m pytest tests/test_gpu_isolation.py -x -q -s --timeout 240 --timeout-method thread > $OUT/iso.txt 2> $OUT/trace.txt || exit $?
