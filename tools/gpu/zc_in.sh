# In-place (zero-copy) latency input: isolation trace with the default
# (in place while bulk uploads are queued), parity with it forced on, and the
# idle 1k latency staged vs in place.  Usage: bash tools/gpu/zc_in.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-zc_in}; mkdir -p $OUT
export TMPDIR=/tmp
SV_STAGE_TRACE=1 SV_LAT_TRACE=1 SV_ISOLATION_OUT=$OUT/isolation_shared.json timeout -k 10 300 python -u -m pytest tests/test_gpu_isolation.py -x -q -s --timeout 240 --timeout-method thread > $OUT/iso.txt 2> $OUT/trace.txt || exit $?
SV_LAT_ZC_IN=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_comb.py tests/test_gpu_longmsg.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity_in_place.txt 2>&1 || exit $?
SV_LAT_ZC_IN=0 AB_ROUNDS=4 timeout -k 10 200 python -u tools/ab_lat_capi.py stellar-core_amd/libstellar_sigverify.so > $OUT/lat_staged.txt 2>&1 || exit $?
SV_LAT_ZC_IN=2 AB_ROUNDS=4 timeout -k 10 200 python -u tools/ab_lat_capi.py stellar-core_amd/libstellar_sigverify.so > $OUT/lat_in_place.txt 2>&1 || exit $?
SV_LAT_ZC_IN=0 AB_ROUNDS=4 timeout -k 10 200 python -u tools/ab_lat_capi.py stellar-core_amd/libstellar_sigverify.so > $OUT/lat_staged2.txt 2>&1 || exit $?
