# Comb kernel: B half of the sum before the hash with the message window
# fetched by LDS-DMA (working tree) vs the committed kernel (variants/
# libsv_prev2.so): latency-path parity, then an interleaved A/B.
# Usage: bash tools/gpu/comb_bfirst.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-comb_bfirst}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_comb.py tests/test_gpu_longmsg.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.txt 2>&1 || exit $?
AB_MODES=warm AB_SIZES=1000,1536,4096 AB_ROUNDS=6 AB_ITERS=300 timeout -k 10 500 python -u tools/ab_lat_capi.py stellar-core_amd/libstellar_sigverify.so ${PREV:-variants/libsv_prev2.so} > $OUT/ab_lat.txt 2>&1 || exit $?
