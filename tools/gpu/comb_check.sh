set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-comb1}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_comb.py -x -v --timeout 150 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
SV_LAT_TRACE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-config1 --no-config35 --no-host-api --latency-iters 100 > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?"
