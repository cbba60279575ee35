# Round 5: the micro-batcher's burst wait (quiet period) on the GPU: the
# integrated tests and the probe grid.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5i}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q -k "scp_integrated or micro_batcher" --timeout 120 --timeout-method thread > $OUT/pytest_scp.txt 2>&1 || exit $?
timeout -k 10 500 python -u tools/scp_probe.py 24000 "1000:5000:0:1:2:4:0:0,1000:5000:0:1:2:4:10:200,1000:5000:0:1:2:4:20:300,1000:5000:0:1:2:4:0:0,1000:5000:0:1:2:4:10:200,1000:5000:0:1:2:4:20:300,4:200:0:1:2:4:10:200,100:500:0:1:2:4:10:200" > $OUT/scp_probe.jsonl 2> $OUT/scp_probe.err || exit $?
