# SHA-512 / BLAKE2b word packing (sv_pack64) A/B: latency through the C-ABI
# (tools/ab_lat_capi.py), 2^20 kernel time (tools/ab_variants.py), then the
# hash-dependent GPU tests.  Usage: bash tools/gpu/ab_sha.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab_sha}; mkdir -p $OUT
export TMPDIR=/tmp
V=variants
AB_ROUNDS=6 AB_ITERS=300 timeout -k 10 400 python -u tools/ab_lat_capi.py $V/libsv_r4head.so $V/libsv_pack64.so > $OUT/ab_lat.txt 2>&1 || exit $?
AB_ROUNDS=8 timeout -k 10 400 python -u tools/ab_variants.py $V/libsv_r4head.so $V/libsv_pack64.so > $OUT/ab_tp.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
