# Latency isolation under bulk load: GPU test (shared mode) + the probe with shared mode off
# usage: bash tools/gpu/iso.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-iso1}; mkdir -p $OUT
SV_ISOLATION_OUT=$OUT/isolation_shared.json timeout -k 10 300 python -u -m pytest tests/test_gpu_isolation.py -x -v -s --timeout 240 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SV_LAT_SHARE_MS=0 timeout -k 10 300 python -u tools/lat_isolation.py --out $OUT/isolation_noshare.json > $OUT/noshare.txt 2>&1
