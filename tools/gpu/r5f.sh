# Round 5: integrated config-4 probe (engine slot released before the
# continuations), the Karatsuba product A/B, the in-process multi-GPU leg
# rehearsed with two device slots on one card.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5f}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q -k "scp_integrated or micro_batcher" --timeout 120 --timeout-method thread > $OUT/pytest_scp.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/scp_probe.py 24000 "1000:5000:0:1:2:4,1000:5000:30:1:2:4,1000:5000:0:1:2:4,1000:5000:30:1:2:4,250:1250:0:1:2:4,100:500:0:1:2:4" > $OUT/scp_probe.jsonl 2> $OUT/scp_probe.err || exit $?
timeout -k 10 120 ./tools/kara_ubench 4000 8 > $OUT/kara_ubench.json 2> $OUT/kara_ubench.err || exit $?
SV_DEVICE_MAP=0,0 timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-latency --no-config1 --no-config35 --no-config4i > $OUT/bench_devmap00.json 2> $OUT/bench_devmap00.err || exit $?
