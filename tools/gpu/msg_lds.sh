# Latency kernels reading each message through an LDS window
# (sv_load_and_hash_lds): GPU parity of the latency paths, the previous kernels
# (variants/libsv_prev.so) vs the current ones at 1000 / 4096 / 12288
# signatures warm and cold, and the comb / octet phase timelines.
# Usage: bash tools/gpu/msg_lds.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-msg_lds}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_comb.py tests/test_gpu_longmsg.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.txt 2>&1 || exit $?
AB_SIZES=1000,2048,4096,12288 AB_ROUNDS=4 AB_ITERS=200 timeout -k 10 500 python -u tools/ab_lat_capi.py stellar-core_amd/libstellar_sigverify.so $V/libsv_prev.so > $OUT/ab_lat.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/comb_phases.py $V/libsv_diag_phases.so > $OUT/phases.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/comb_phases.py --octet $V/libsv_diag_ophases.so > $OUT/ophases.txt 2>&1 || exit $?
