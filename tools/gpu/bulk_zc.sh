# One-chunk host batches read in place (SV_BULK_ZC_IN=1, default) vs staged
# (0), alternating processes, plus the GPU suite parts that exercise the host
# staging.  Usage: bash tools/gpu/bulk_zc.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-bulk_zc}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py tests/test_gpu_keytables.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit $?
for r in 1 2 3; do
  for m in 0 1; do
    SV_BULK_ZC_IN=$m timeout -k 10 200 python -u tools/host_api_sizes.py 30 >> $OUT/sizes_m$m.jsonl 2> $OUT/err_m${m}_r$r.txt || exit $?
  done
done
