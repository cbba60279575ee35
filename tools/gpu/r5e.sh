# Round 5: GPU suite + the integrated config-4 probe (LDS-DMA window staging) after the lane's cache
# keys moved to an LDS-staged kernel on a side stream.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5e}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/scp_probe.py 12000 "1000:5000:0:1:2:4,1000:5000:30:1:2:4,1000:5000:100:1:2:4,1000:5000:0:2:2:4,1000:5000:0:1:1:1,250:1250:0:1:2:4,100:500:0:1:2:4" > $OUT/scp_probe.jsonl 2> $OUT/scp_probe.err || exit $?
SV_HOST_TRACE=1 SV_LAT_TRACE=1 timeout -k 10 300 python -u tools/scp_probe.py 6000 "1000:5000:0:1:2:4" > $OUT/scp_trace.jsonl 2> $OUT/scp_trace.err || exit $?
